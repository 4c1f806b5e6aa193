// The fp32 PPO update's Linear forward and input-gradient GEMMs on the matrix cores (include/t1policy.h,
// t1policy_gemm_nt_f32): C[r, n] = sum_k A[r, k] B[n, k] (+ bias[n]) (then ELU, alpha 1) for row-major fp32 A (R x K)
// and B (N x K) -- what nn.Linear's forward (y = x W^T + b, B = W) and its input gradient (gx = gy W, B = W^T) compute for
// every layer of actor_critic_dh.py:45-111 in the update (dh_ppo.py:155-182), at the reference's fp32 precision.
//
// hipBLASLt's fp32 GEMMs run on the fp32 matrix rate (~157 TFLOP/s dense).  Here each fp32 operand is split into three
// bf16 parts, v = v1 + v2 + v3 (v1 = bf16(v), v2 = bf16(v - v1), v3 = bf16(v - v1 - v2): 24+ significant bits), and a
// product is the six part products down to 2^-16 of |a b| (the three dropped ones lie below 2^-24), each exact in fp32
// and accumulated by v_mfma_f32_32x32x16_bf16 in fp32: fp32-class sums at the bf16 rate / 6 (~415 TFLOP/s dense).
//
// A workgroup owns a 128 x 128 output tile; four waves own 64 x 64 quarters (2 x 2 accumulators).  Both operands have
// the reduction index k contiguous, so a fragment (a lane holds 8 consecutive k of one row / column) is two ds_read_b128
// of a row-major staged chunk; the chunk is 32 k wide (two k-steps), staged as fp32 (pitch 36 words), double-buffered,
// with the next two chunks' loads in flight in registers (issued unconditionally at clamped indices; the staging stores
// zero what lies outside the matrix).  The parts are formed from the fragments (VALU, in the MFMAs' shadow).
// Deterministic: one fixed summation order per output (k ascending), no atomics.
// Measured (tools/wgrad_bench.py --f32, the update's 15 layers at 49,152 rows): forward 876-904 us per minibatch against
// hipBLASLt's addmm 873-883, input gradient 883-931 against mm 931-933 (profiles/r06f_*, r06j_*); forming the parts once
// per staged element (three bf16 images, one ds_read_b128 per fragment part) measured 922 / 973 us and was removed: the
// split's VALU is not what bounds it.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr int GM_T = 128;          // output tile (rows and columns)
constexpr int GM_KC = 32;          // k per staged chunk (two k-steps of 16)
constexpr int GM_PITCH = GM_KC + 4;  // fp32 words per staged row
constexpr int GM_LPT = GM_T * GM_KC / 256;  // loads per thread per operand per chunk: 16

struct GmStage {
  float v[GM_LPT];
};
// thread t loads k = k0 + (t & 31) of rows r0 + (t >> 5) + 8 i (a wave instruction: two rows x 128 B), clamped
__device__ __forceinline__ void gm_load(const float* __restrict__ z, int rows, int K, int r0, int k0, int t,
                                        GmStage& v) {
  const int k = k0 + (t & 31);
  const int kc = k < K ? k : K - 1;
#pragma unroll
  for (int i = 0; i < GM_LPT; ++i) {
    const int r = r0 + (t >> 5) + 8 * i;
    v.v[i] = z[(size_t)(r < rows ? r : rows - 1) * K + kc];
  }
}
__device__ __forceinline__ void gm_store(float* img, int rows, int K, int r0, int k0, int t, const GmStage& v) {
  const bool k_ok = k0 + (t & 31) < K;
#pragma unroll
  for (int i = 0; i < GM_LPT; ++i) {
    const int rr = (t >> 5) + 8 * i;
    img[rr * GM_PITCH + (t & 31)] = (k_ok && r0 + rr < rows) ? v.v[i] : 0.0f;
  }
}
struct Bf3 {
  bf8 p[3];
};
// rows row0 + (lane & 31), k = 16 ks + 8 (lane >> 5) .. + 7 of a staged chunk, split in three bf16 parts
__device__ __forceinline__ void gm_frag(const float* img, int ks, int row0, int lane, Bf3& f) {
  const float* p = img + (row0 + (lane & 31)) * GM_PITCH + 16 * ks + 8 * (lane >> 5);
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 h1 = (__bf16)v[j];
    const float r1 = v[j] - (float)h1;
    const __bf16 h2 = (__bf16)r1;
    f.p[0][j] = h1;
    f.p[1][j] = h2;
    f.p[2][j] = (__bf16)(r1 - (float)h2);
  }
}
__device__ __forceinline__ f16v mfma_bf3(const Bf3& a, const Bf3& b, f16v acc) {  // the smallest products first
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[2], b.p[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[1], b.p[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[0], b.p[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[1], b.p[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[0], b.p[1], acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[0], b.p[0], acc, 0, 0, 0);
}

// grid.x: row tiles, grid.y: column tiles.  act: 0 none, 1 ELU (alpha 1, the policy's nn.ELU), 2 times ELU's derivative
// at the ELU outputs aux (R x N): the input gradient of a Linear whose input is an ELU's output
__global__ __launch_bounds__(256, 2) void k_gemm_nt_f32x3(const float* __restrict__ A, const float* __restrict__ B,
                                                          const float* __restrict__ bias, const float* __restrict__ aux,
                                                          float* __restrict__ C, int R, int N, int K, int act) {
  __shared__ __attribute__((aligned(16))) float IMG[2][2][GM_T * GM_PITCH];  // [buffer][A, B]
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, h = lane >> 5;
  const int wm = wave & 1, wn = wave >> 1;
  const int r0 = GM_T * blockIdx.x, n0 = GM_T * blockIdx.y;
  const int m_rem = R - (r0 + 64 * wm), n_rem = N - (n0 + 64 * wn);
  const int mb_n = m_rem <= 0 ? 0 : (m_rem > 32 ? 2 : 1), nb_n = n_rem <= 0 ? 0 : (n_rem > 32 ? 2 : 1);
  f16v acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.0f;
  // one chunk's loads in flight in registers while the previous one multiplies (two LDS buffers, one barrier per chunk)
  GmStage va, vb;
  gm_load(A, R, K, r0, 0, t, va);
  gm_load(B, N, K, n0, 0, t, vb);
  int buf = 0;
  auto chunk = [&](GmStage& ra, GmStage& rb, int k0) {
    gm_store(IMG[buf][0], R, K, r0, k0, t, ra);
    gm_store(IMG[buf][1], N, K, n0, k0, t, rb);
    gm_load(A, R, K, r0, k0 + GM_KC, t, ra);
    gm_load(B, N, K, n0, k0 + GM_KC, t, rb);
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
    if (mb_n > 0 && nb_n > 0) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        Bf3 fa[2], fb[2];
#pragma unroll
        for (int a = 0; a < 2; ++a) gm_frag(IMG[buf][0], ks, 64 * wm + 32 * a, lane, fa[a]);
#pragma unroll
        for (int b = 0; b < 2; ++b) gm_frag(IMG[buf][1], ks, 64 * wn + 32 * b, lane, fb[b]);
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          if (a >= mb_n) break;
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            if (b >= nb_n) break;
            acc[a][b] = mfma_bf3(fa[a], fb[b], acc[a][b]);
          }
        }
      }
    }
    buf ^= 1;
  };
  for (int k0 = 0; k0 < K; k0 += GM_KC) chunk(va, vb, k0);
  // C/D of a 32 x 32 tile: column n = lane & 31, row m = (q & 3) + 8 (q >> 2) + 4 h
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    if (a >= mb_n) break;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      if (b >= nb_n) break;
      const int n = n0 + 64 * wn + 32 * b + (lane & 31);
      const float bv = (bias != nullptr && n < N) ? bias[n] : 0.0f;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int m = r0 + 64 * wm + 32 * a + (q & 3) + 8 * (q >> 2) + 4 * h;
        float v = acc[a][b][q] + bv;
        if (act == 1) v = v > 0.0f ? v : expm1f(v);
        if (m < R && n < N) {
          if (act == 2) {  // times ELU's derivative at the ELU output e (alpha 1: 1 for e > 0, else e + 1)
            const float e = aux[(size_t)m * N + n];
            v = v * (e > 0.0f ? 1.0f : e + 1.0f);
          }
          C[(size_t)m * N + n] = v;
        }
      }
    }
  }
}

}  // namespace

extern "C" {

int t1policy_gemm_nt_f32(const float* A, const float* B, const float* bias, const float* aux, float* C, int R, int N,
                         int K, int act, void* stream) {
  if (!A || !B || !C || R <= 0 || N <= 0 || K <= 0 || act < 0 || act > 2 || (act == 2 && !aux)) return -1;
  if ((long long)R * (K > N ? K : N) >= (1LL << 31)) return -1;
  const dim3 grid((R + GM_T - 1) / GM_T, (N + GM_T - 1) / GM_T);
  hipLaunchKernelGGL(k_gemm_nt_f32x3, grid, dim3(256), 0, (hipStream_t)stream, A, B, bias, aux, C, R, N, K, act);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
