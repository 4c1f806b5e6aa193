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
// the reduction index k contiguous, so a fragment (a lane holds 8 consecutive k of one row / column) is one ds_read_b128
// per part.  The product kernel, k_gemm_nt_f32x3s (below), splits each element into its parts ONCE, as it stages it
// (three bf16 LDS images per operand, 16 k per chunk), runs each chunk's 24 MFMAs in two halves beside the next chunk's
// split + stores and fragment reads, loads two chunks ahead through a buffer descriptor (16-B loads, rows past the matrix
// read 0), and walks the output tiles XCD by XCD so the column tiles of a row tile share its HBM read.
// Deterministic: one fixed summation order per output (k ascending), no atomics.
// Measured (tools/probes/gemm_whatif.hip, 49,152 rows; profiles/r06n_gemm_*): 98-101 us at N 256 / K 512 against 122 for
// the first form (k_gemm_nt_f32x3, parts formed per fragment by each of the two waves that read it), 131 against 158 at
// 302 / 512, 118 against 149 at 256 / 768, 128 against 146 at 768 / 219.  What-if builds put the rest on the additive
// cost of the MFMAs (~53 us alone at 256 / 512), the staging (~33) and the loads (~25): the SIMD overlaps little of it.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <type_traits>

namespace {

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

#ifndef T1_GEMM_WHATIF  // timing-only what-if builds (tools/probes/gemm_whatif.hip): bit 0 no in-loop global loads,
#define T1_GEMM_WHATIF 0  // bit 1 no LDS stores, bit 2 one MFMA per product, bit 3 no split (v1 only)
#endif
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
#if T1_GEMM_WHATIF & 8
#pragma unroll
  for (int j = 0; j < 8; ++j) f.p[0][j] = f.p[1][j] = f.p[2][j] = (__bf16)v[j];
  return;
#endif
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

// ELU (alpha 1) without the libm expm1f call in the epilogue: expm1(v) for v <= 0 as a degree-10 Taylor polynomial on
// [-1, 0] (truncation below 2.5e-8 of 1 / 11!, relative to |expm1| >= 0.63 |v| there) and exp(v) - 1 below -1 (no
// cancellation: |result| > 0.63); max error a few ulp of the result, against torch's expm1 ELU (tests: 2e-6)
__device__ __forceinline__ float elu1(float v) {
  if (v > 0.0f) return v;
  float p = 1.0f / 39916800.0f;  // 1 / 11!
  p = fmaf(p, v, 1.0f / 3628800.0f);
  p = fmaf(p, v, 1.0f / 362880.0f);
  p = fmaf(p, v, 1.0f / 40320.0f);
  p = fmaf(p, v, 1.0f / 5040.0f);
  p = fmaf(p, v, 1.0f / 720.0f);
  p = fmaf(p, v, 1.0f / 120.0f);
  p = fmaf(p, v, 1.0f / 24.0f);
  p = fmaf(p, v, 1.0f / 6.0f);
  p = fmaf(p, v, 0.5f);
  p = fmaf(p, v, 1.0f);
  const float poly = p * v;
  return v >= -1.0f ? poly : __expf(v) - 1.0f;
}

// C/D of a 32 x 32 tile: column n = lane & 31, row m = (q & 3) + 8 (q >> 2) + 4 h
__device__ __forceinline__ void gm_epilogue(const f16v (&acc)[2][2], const float* __restrict__ bias,
                                            const float* __restrict__ aux, float* __restrict__ C, int R, int N, int r0,
                                            int n0, int wm, int wn, int mb_n, int nb_n, int lane, int act) {
  const int h = lane >> 5;
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    if (a >= mb_n) break;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      if (b >= nb_n) break;
      const int n = n0 + 64 * wn + 32 * b + (lane & 31);
      const float bv = (bias != nullptr && n < N) ? bias[n] : 0.0f;
      // act 2: the tile's 16 ELU outputs loaded together first (clamped in-matrix, unconditional: all in flight)
      float e[16];
      if (act == 2) {
        const int nc = n < N ? n : N - 1;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int m = r0 + 64 * wm + 32 * a + (q & 3) + 8 * (q >> 2) + 4 * h;
          e[q] = aux[(size_t)(m < R ? m : R - 1) * N + nc];
        }
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int m = r0 + 64 * wm + 32 * a + (q & 3) + 8 * (q >> 2) + 4 * h;
        float v = acc[a][b][q] + bv;
        if (act == 1) v = elu1(v);
        // act 2: times ELU's derivative at the ELU output e (alpha 1: 1 for e > 0, else e + 1)
        if (act == 2) v = v * (e[q] > 0.0f ? 1.0f : e[q] + 1.0f);
        if (m < R && n < N) C[(size_t)m * N + n] = v;
      }
    }
  }
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
    if (!(T1_GEMM_WHATIF & 2)) {
      gm_store(IMG[buf][0], R, K, r0, k0, t, ra);
      gm_store(IMG[buf][1], N, K, n0, k0, t, rb);
    }
    if (!(T1_GEMM_WHATIF & 1) || k0 == 0) gm_load(A, R, K, r0, k0 + GM_KC, t, ra);
    if (!(T1_GEMM_WHATIF & 1) || k0 == 0) gm_load(B, N, K, n0, k0 + GM_KC, t, rb);
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
            if (T1_GEMM_WHATIF & 4)
              acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a].p[0], fb[b].p[0], acc[a][b], 0, 0, 0);
            else
              acc[a][b] = mfma_bf3(fa[a], fb[b], acc[a][b]);
          }
        }
      }
    }
    buf ^= 1;
  };
  for (int k0 = 0; k0 < K; k0 += GM_KC) chunk(va, vb, k0);
  gm_epilogue(acc, bias, aux, C, R, N, r0, n0, wm, wn, mb_n, nb_n, lane, act);
}

constexpr int GP_OOB = 0x40000000;  // a byte offset past every operand's num_records (buffer loads read 0 there)

// ---- the staged-split form (the default; T1_GEMM_STAGED=0 selects the first form above): each fp32 element is split into its three bf16 parts ONCE, by the
// thread that stages it, instead of by each of the two waves that read it as a fragment, and the parts go to three bf16
// LDS images that the fragments read back directly (ds_read_b128, no VALU between the LDS and the MFMAs).  One k-step
// (16 k) per staged chunk: a chunk's 24 MFMAs run as two halves of 12, the first beside the split + stores of the next
// chunk and the loads of the one after, the second beside the reads of the next chunk's fragments; one barrier per
// chunk between the halves.  Rows are 16 k + 8 pad bf16 (48 B): the b128 fragment reads are conflict-free.
constexpr int GS_KC = 16, GS_PITCH = 24;
constexpr int GS_IMG = GM_T * GS_PITCH;  // bf16 per part image
typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
// thread t stages k = k0 + 4 (t & 3) .. + 3 of rows (t >> 2) and (t >> 2) + 64: one 16-B load per row (4-B aligned
// at an odd K: unaligned 16-B loads are exact on gfx950, tools/probes/unaligned_x4.hip), rows past the matrix reading 0
// through the descriptor's range check; the chunk that crosses K (uniform) takes 4-B loads, each past K reading 0
template <bool FULL>  // FULL: the chunk lies inside K (a uniform fact the caller knows; no branch in the main loop)
__device__ __forceinline__ void gs_load(__amdgpu_buffer_rsrc_t rs, int base, int row64, int K, int k0, int kq,
                                        f4 (&v)[2]) {
  if (FULL || k0 + GS_KC <= K) {
    v[0] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, base + 4 * k0, 0, 0));
    v[1] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, base + 4 * k0 + row64, 0, 0));
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int vo = k0 + kq + j < K ? base + 4 * (k0 + j) : GP_OOB;
      v[0][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, vo, 0, 0));
      v[1][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, vo + row64, 0, 0));
    }
  }
}
// the three parts of 4 values into the part images (one ds_write_b64 per part and row)
__device__ __forceinline__ void gs_split_store(__bf16* img, int row, int kq, f4 v) {
  bf4 p1, p2, p3;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const __bf16 h1 = (__bf16)v[j];
    const float r1 = v[j] - (float)h1;
    const __bf16 h2 = (__bf16)r1;
    p1[j] = h1;
    p2[j] = h2;
    p3[j] = (__bf16)(r1 - (float)h2);
  }
  const int o = row * GS_PITCH + kq;
  *reinterpret_cast<bf4*>(img + o) = p1;
  *reinterpret_cast<bf4*>(img + GS_IMG + o) = p2;
  *reinterpret_cast<bf4*>(img + 2 * GS_IMG + o) = p3;
}
// rows row0 + (lane & 31), k = 8 (lane >> 5) .. + 7 of a staged chunk's three part images
__device__ __forceinline__ void gs_frag(const __bf16* img, int row0, int lane, Bf3& f) {
  const int o = (row0 + (lane & 31)) * GS_PITCH + 8 * (lane >> 5);
#pragma unroll
  for (int p = 0; p < 3; ++p) f.p[p] = *reinterpret_cast<const bf8*>(img + p * GS_IMG + o);
}
struct GsFrags {
  Bf3 a[2], b[2];
};
// grid: 8 x per_xcd workgroups (1-D).  Workgroup i runs on XCD i mod 8 and takes output tile q = (i mod 8) per_xcd +
// i / 8 (column tiles fastest): an XCD works through a contiguous run of tiles, so the column tiles of one row tile run
// on the same XCD at about the same time and read that row tile of A from HBM once (the other reads hit its L2)
// B given as [K][N] (BKN, ldb >= N): thread t stages column n0 + (t & 127) of the 8 k-rows k0 + 8 (t >> 7) .. + 7 (each
// wave load is 64 consecutive columns of one k-row), so it holds 8 consecutive k of one column and stores each part
// with one ds_write_b128 -- the transposed weight of an input gradient (gx = g W: B = W^T) read in place
__device__ __forceinline__ void gs_load_kn(__amdgpu_buffer_rsrc_t rs, int base, int rowb, int k0, f4 (&v)[2]) {
#pragma unroll
  for (int i = 0; i < 8; ++i)
    v[i >> 2][i & 3] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, base + (k0 + i) * rowb, 0, 0));
}
__device__ __forceinline__ void gs_split_store8(__bf16* img, int col, int g, const f4 (&v)[2]) {
  bf8 p1, p2, p3;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float x = v[j >> 2][j & 3];
    const __bf16 h1 = (__bf16)x;
    const float r1 = x - (float)h1;
    const __bf16 h2 = (__bf16)r1;
    p1[j] = h1;
    p2[j] = h2;
    p3[j] = (__bf16)(r1 - (float)h2);
  }
  const int o = col * GS_PITCH + 8 * g;
  *reinterpret_cast<bf8*>(img + o) = p1;
  *reinterpret_cast<bf8*>(img + GS_IMG + o) = p2;
  *reinterpret_cast<bf8*>(img + 2 * GS_IMG + o) = p3;
}
// NARROW (N <= 64, e.g. the 16-channel history layer over 294,912 rows): the MFMAs of 32 x 32 tiles past N are skipped
// (wave-uniform branches; at N <= 64 the waves of the second column half have no tile at all).  lda / ldb: the row
// strides of A ([R][lda]) and B ([N][ldb], or [K][ldb] under BKN), in elements
template <bool NARROW, bool BKN>
__global__ __launch_bounds__(256, 2) void k_gemm_nt_f32x3s(const float* __restrict__ A, int lda, const float* __restrict__ B,
                                                           int ldb, const float* __restrict__ bias,
                                                           const float* __restrict__ aux, float* __restrict__ C, int R,
                                                           int N, int K, int act, int col_tiles, int per_xcd) {
  __shared__ __attribute__((aligned(16))) __bf16 IMG[2][2][3 * GS_IMG];  // [buffer][A, B][part][row][k]
  const int q = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  if (q >= col_tiles * ((R + GM_T - 1) / GM_T)) return;  // the last XCD's spare workgroups (uniform)
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int r0 = GM_T * (q / col_tiles), n0 = GM_T * (q % col_tiles);
  const int m_rem = R - (r0 + 64 * wm), n_rem = N - (n0 + 64 * wn);
  const int mb_n = m_rem <= 0 ? 0 : (m_rem > 32 ? 2 : 1), nb_n = n_rem <= 0 ? 0 : (n_rem > 32 ? 2 : 1);
  // num_records: through the last element (rows past the matrix, and under BKN k-rows past K, read 0)
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(A), 0, ((R - 1) * lda + K) * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(B), 0, (BKN ? (K - 1) * ldb + N : (N - 1) * ldb + K) * 4, 0x00020000);
  const int kq = 4 * (t & 3), srow = t >> 2, arow64 = 64 * lda * 4, brow64 = 64 * ldb * 4;
  const int ba = ((r0 + srow) * lda + kq) * 4;
  const int bcol = t & 127, bg = t >> 7;  // BKN staging
  const int bb = BKN ? (n0 + bcol < N ? (8 * bg * ldb + n0 + bcol) * 4 : GP_OOB) : ((n0 + srow) * ldb + kq) * 4;
  f16v acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.0f;
  const int nch = (K + GS_KC - 1) / GS_KC;
  // loads two chunks ahead: register slot j & 1 holds chunk j from its load (two iterations before it is staged)
  f4 va[2][2], vb[2][2];
  auto load = [&](int slot, int k0, auto full) {
    gs_load<decltype(full)::value>(ra, ba, arow64, K, k0, kq, va[slot]);
    if constexpr (BKN)
      gs_load_kn(rb, bb, ldb * 4, k0, vb[slot]);
    else
      gs_load<decltype(full)::value>(rb, bb, brow64, K, k0, kq, vb[slot]);
  };
  using Full = std::integral_constant<bool, true>;
  using Edge = std::integral_constant<bool, false>;
  auto stage = [&](int buf, int slot) {
    gs_split_store(IMG[buf][0], srow, kq, va[slot][0]);
    gs_split_store(IMG[buf][0], srow + 64, kq, va[slot][1]);
    if constexpr (BKN) {
      gs_split_store8(IMG[buf][1], bcol, bg, vb[slot]);
    } else {
      gs_split_store(IMG[buf][1], srow, kq, vb[slot][0]);
      gs_split_store(IMG[buf][1], srow + 64, kq, vb[slot][1]);
    }
  };
  auto frags = [&](int buf, GsFrags& f) {
#pragma unroll
    for (int b = 0; b < 2; ++b) gs_frag(IMG[buf][1], 64 * wn + 32 * b, lane, f.b[b]);
#pragma unroll
    for (int a = 0; a < 2; ++a) gs_frag(IMG[buf][0], 64 * wm + 32 * a, lane, f.a[a]);
  };
  load(0, 0, Edge());
  load(1, GS_KC, Edge());
  stage(0, 0);
  load(0, 2 * GS_KC, Edge());
  __syncthreads();
  GsFrags f0, f1;
  frags(0, f0);
  // chunk c (fragments in fc, image buffer c & 1): the first half of its MFMAs beside staging chunk c + 1 (slot
  // (c + 1) & 1) and loading chunk c + 3 into that slot; barrier; the second half beside reading chunk c + 1's
  // fragments into fn
#ifndef T1_GEMM_S_WHATIF  // timing-only what-if builds (tools/probes/gemm_whatif.hip): bit 0 no barrier, 1 no staging,
#define T1_GEMM_S_WHATIF 0  // 2 no fragment reads, 3 no loads, 4 one MFMA per product
#endif
  auto mf = [&](int a, int b, const GsFrags& f) {
    if (NARROW && (a >= mb_n || b >= nb_n)) return;
    if (T1_GEMM_S_WHATIF & 16)
      acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[a].p[0], f.b[b].p[0], acc[a][b], 0, 0, 0);
    else
      acc[a][b] = mfma_bf3(f.a[a], f.b[b], acc[a][b]);
  };
  auto iter = [&](int c, int slot, GsFrags& fc, GsFrags& fn, auto full) {
    const int nxt = (c + 1) & 1;
    __builtin_amdgcn_sched_barrier(0);
    if (!(T1_GEMM_S_WHATIF & 2)) stage(nxt, slot);
    if (!(T1_GEMM_S_WHATIF & 8)) load(slot, (c + 3) * GS_KC, full);
    mf(0, 0, fc);
    mf(0, 1, fc);
#if !T1_GEMM_NO_SCHED
    // the MFMAs from the start of the segment, the split between them
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
      __builtin_amdgcn_sched_group_barrier(0x002, 8, 1);
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 1);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 1);
    }
#endif
    __builtin_amdgcn_sched_barrier(0);
    if (!(T1_GEMM_S_WHATIF & 1)) __syncthreads();
    if (!(T1_GEMM_S_WHATIF & 4)) frags(nxt, fn);
    mf(1, 0, fc);
    mf(1, 1, fc);
#if !T1_GEMM_NO_SCHED
    // the next chunk's fragment reads first: their latency runs under these 12 MFMAs
    __builtin_amdgcn_sched_group_barrier(0x100, 12, 2);
    __builtin_amdgcn_sched_group_barrier(0x008, 12, 2);
#endif
  };
  // main loop while both iterations' loads (chunks c + 3, c + 4) lie inside K, then the edge iterations
  const int nfull = K / GS_KC;
  int c = 0;
  for (; c + 4 < nfull; c += 2) {
    iter(c, 1, f0, f1, Full());
    iter(c + 1, 0, f1, f0, Full());
  }
  for (; c + 1 < nch; c += 2) {
    iter(c, 1, f0, f1, Edge());
    iter(c + 1, 0, f1, f0, Edge());
  }
  if (c < nch) iter(c, 1, f0, f1, Edge());
  __builtin_amdgcn_sched_barrier(0);
  gm_epilogue(acc, bias, aux, C, R, N, r0, n0, wm, wn, mb_n, nb_n, lane, act);
}
// T1_GEMM_STAGED (A/B): 1 (default) k_gemm_nt_f32x3s; 0 the first form, k_gemm_nt_f32x3 (parts formed per fragment)
bool gemm_staged() {
  static const bool v = [] {
    const char* e = getenv("T1_GEMM_STAGED");
    return !(e && e[0] == '0');
  }();
  return v;
}

}  // namespace

extern "C" {

int t1policy_gemm_f32(const float* A, int lda, const float* B, int ldb, int b_kn, const float* bias, const float* aux,
                      float* C, int R, int N, int K, int act, void* stream) {
  if (!A || !B || !C || R <= 0 || N <= 0 || K <= 0 || act < 0 || act > 2 || (act == 2 && !aux)) return -1;
  if (lda < K || ldb < (b_kn ? N : K)) return -1;
  // every byte offset below GP_OOB (the descriptors' 32-bit offsets; 1 GiB per operand)
  if ((long long)R * lda * 4 >= GP_OOB || (long long)(b_kn ? K : N) * ldb * 4 >= GP_OOB ||
      (long long)R * N >= (1LL << 31))
    return -1;
  const int row_tiles = (R + GM_T - 1) / GM_T, col_tiles = (N + GM_T - 1) / GM_T;
  const int tiles = row_tiles * col_tiles, per_xcd = (tiles + 7) / 8;
  const dim3 grid(8 * per_xcd), blk(256);
  hipStream_t st = (hipStream_t)stream;
  if (N <= 64 && b_kn)
    hipLaunchKernelGGL((k_gemm_nt_f32x3s<true, true>), grid, blk, 0, st, A, lda, B, ldb, bias, aux, C, R, N, K, act,
                       col_tiles, per_xcd);
  else if (N <= 64)
    hipLaunchKernelGGL((k_gemm_nt_f32x3s<true, false>), grid, blk, 0, st, A, lda, B, ldb, bias, aux, C, R, N, K, act,
                       col_tiles, per_xcd);
  else if (b_kn)
    hipLaunchKernelGGL((k_gemm_nt_f32x3s<false, true>), grid, blk, 0, st, A, lda, B, ldb, bias, aux, C, R, N, K, act,
                       col_tiles, per_xcd);
  else
    hipLaunchKernelGGL((k_gemm_nt_f32x3s<false, false>), grid, blk, 0, st, A, lda, B, ldb, bias, aux, C, R, N, K, act,
                       col_tiles, per_xcd);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int t1policy_gemm_nt_f32(const float* A, const float* B, const float* bias, const float* aux, float* C, int R, int N,
                         int K, int act, void* stream) {
  if (!A || !B || !C || R <= 0 || N <= 0 || K <= 0 || act < 0 || act > 2 || (act == 2 && !aux)) return -1;
  if ((long long)R * (K > N ? K : N) >= (1LL << 31)) return -1;
  const bool fits = (long long)R * K * 4 < GP_OOB && (long long)N * K * 4 < GP_OOB;
  if (gemm_staged() && fits) return t1policy_gemm_f32(A, K, B, K, 0, bias, aux, C, R, N, K, act, stream);
  const dim3 grid((R + GM_T - 1) / GM_T, (N + GM_T - 1) / GM_T);
  hipLaunchKernelGGL(k_gemm_nt_f32x3, grid, dim3(256), 0, (hipStream_t)stream, A, B, bias, aux, C, R, N, K, act);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
