// The DH policy's first history conv in the PPO update under the opt-in bf16 update (include/t1policy.h,
// t1policy_conv1_*_bf16): forward and weight gradient on the matrix cores, straight from the (B, 66, 47) bf16
// observation history -- no unfolded (B x 14, 396) copy.
//
// The reference's layer (actor_critic_dh.py:83-96): nn.Conv1d(66 -> 32, kernel 6, stride 3) over the 47 features of
// the 66 frames.  The build's autograd path ran it as unfold + GEMM (dh_policy.conv1d_as_gemm): at the update's
// 49,152-sample minibatch a 545 MB unfold copy (310 us), a 688k x 396 GEMM (121 us) and a split-K weight-gradient
// bmm + sum (199 + 32 us) per minibatch (profiles/r04p2_ppo_update_profile_bf16_eager.txt).  Here:
//
//   k_conv1_fwd_bf16    y[b, l, o] = bf16(bias[o] + sum_{c,t} w[o, c, t] x[b, c, 3 l + t]): per sample a (14 x 396) .
//                       (396 x 32) product on v_mfma_f32_16x16x32_bf16 -- the inference conv's K order (8 slots per
//                       channel: its 6 taps and 2 zeros, so a lane's A fragment is 6 contiguous inputs), the bf16
//                       weight fragments in registers, each wave streaming a contiguous run of samples through its own
//                       LDS rows.  As autocast's addmm: bf16 operands, fp32 accumulation, bias added as bf16 then one
//                       rounding of the sum to bf16.
//   k_conv1_wgrad_bf16  gW[o, c, t] = sum_{b, l} gy[b, l, o] x[b, c, 3 l + t], gb[o] = sum gy: per sample ONE k-step of
//                       v_mfma_f32_32x32x16_bf16 (k = the 14 output positions + 2 zero rows) for each of the 13 32-column
//                       tiles of the 396 (c, t) columns; a workgroup accumulates a run of samples in registers and
//                       stores one fp32 partial; k_conv1_wgrad_reduce sums the partials in a fixed tree
//                       (deterministic, so eager and graph-replayed updates stay bit-identical).
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr int TC_C = 66, TC_L = 47, TC_O = 32, TC_K = 6, TC_S = 3, TC_LOUT = 14;
constexpr int TC_STEPS = 17;                     // forward K-steps of 32: 4 channels each (66 + 2 zero channels)
constexpr int TC_CPAD = 4 * TC_STEPS;            // 68 staged channel rows
constexpr int TC_SAMPLE = TC_C * TC_L;           // 3,102 bf16 per sample
constexpr int TC_FRAG_BYTES = TC_STEPS * 2 * 64 * 16;  // [step][column tile][lane] bf8: 34,816
constexpr int TC_COLS = TC_C * TC_K;             // 396 weight-gradient columns (c, t)
constexpr int TC_CT = (TC_COLS + 31) / 32;       // 13 column tiles of 32
constexpr int TC_PART = TC_O * TC_CT * 32 + TC_O;  // partial floats per workgroup: 32 x 416 + 32 bias
constexpr int TC_WG_BLOCKS = 512;                // weight-gradient workgroups (partials)

__device__ __forceinline__ uint16_t bf16_bits(float v) {  // round to nearest even, as torch's .to(torch.bfloat16)
  const uint32_t u = __float_as_uint(v);
  if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)((u >> 16) | ((u & 0xffffu) ? 0x40u : 0u));  // inf / nan
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float bf16_float(uint16_t b) { return __uint_as_float((uint32_t)b << 16); }

// ---- forward weight fragments: lane l of (step s, column tile nt) holds B[k = 8 (l >> 4) + j][n = l & 15] =
// bf16(w[o = 16 nt + (l & 15)][c = 4 s + (l >> 4)][t = j]) for j < 6, else 0 (the layout of t1policy.hip's fragments)
__global__ __launch_bounds__(256) void k_conv1_pack_bf16(const float* __restrict__ w, uint16_t* __restrict__ frag) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= TC_STEPS * 2 * 64) return;
  const int s = e >> 7, nt = (e >> 6) & 1, l = e & 63;
  const int c = 4 * s + (l >> 4), o = 16 * nt + (l & 15);
#pragma unroll
  for (int j = 0; j < 8; ++j)
    frag[(size_t)e * 8 + j] = (c < TC_C && j < TC_K) ? bf16_bits(w[(o * TC_C + c) * TC_K + j]) : (uint16_t)0;
}

// One wave per SIMD, four waves per workgroup, each wave a contiguous run of samples staged in its own LDS rows
// (the next two samples' loads in flight while the current one multiplies).
constexpr int TF_WAVES = 4;
constexpr int TF_PER_LANE = (TC_SAMPLE / 2 + 63) / 64;  // 25 32-bit words per lane (1,551 per sample)
__global__ __launch_bounds__(64 * TF_WAVES) __attribute__((amdgpu_waves_per_eu(1, 2)))
void k_conv1_fwd_bf16(const uint16_t* __restrict__ x, const bf8* __restrict__ frag, const float* __restrict__ bias,
                      uint16_t* __restrict__ y, int batch) {
  __shared__ uint32_t XS[TF_WAVES][TC_CPAD * TC_L / 2 + 1];  // bf16 pairs; channels 66, 67 stay zero
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = blockIdx.x * TF_WAVES + wave, nw = gridDim.x * TF_WAVES;
  const int b0 = (int)((long long)g * batch / nw), b1 = (int)((long long)(g + 1) * batch / nw);
  uint32_t* X = XS[wave];
  for (int i = TC_SAMPLE / 2 + lane; i < TC_CPAD * TC_L / 2 + 1; i += 64) X[i] = 0u;
  bf8 bfr[TC_STEPS][2];
#pragma unroll
  for (int s = 0; s < TC_STEPS; ++s)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) bfr[s][nt] = frag[(s * 2 + nt) * 64 + lane];
  float bo[2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) bo[nt] = bf16_float(bf16_bits(bias[16 * nt + (lane & 15)]));
  const uint32_t* xw = reinterpret_cast<const uint32_t*>(x);  // a sample is 6,204 B: 4-byte aligned
  if (b0 >= b1) return;  // an empty run (batch below the wave count); the kernel has no workgroup barrier
  // two samples' loads in flight (register slots pa, pb); a slot is refilled with the sample two ahead (past the run:
  // the run's last sample again, an L2 hit) as soon as it is staged, unconditionally, so each wait counts only that
  // slot's loads
  uint32_t pa[TF_PER_LANE], pb[TF_PER_LANE];
  auto load = [&](uint32_t (&p)[TF_PER_LANE], int bs) {
    const uint32_t* src = xw + (size_t)(bs < b1 ? bs : b1 - 1) * (TC_SAMPLE / 2);
#pragma unroll
    for (int k = 0; k < TF_PER_LANE; ++k) {
      const int i = lane + 64 * k;
      p[k] = src[i < TC_SAMPLE / 2 ? i : TC_SAMPLE / 2 - 1];
    }
  };
  load(pa, b0);
  __builtin_amdgcn_sched_barrier(0);
  load(pb, b0 + 1);
  __builtin_amdgcn_sched_barrier(0);
  const int r = lane & 15, kg = lane >> 4;
  const int rr = r < TC_LOUT ? r : TC_LOUT - 1;  // rows 14, 15: row 13's inputs, never stored
  const uint16_t* Xh = reinterpret_cast<const uint16_t*>(X);
  auto process = [&](uint32_t (&p)[TF_PER_LANE], int b) {
#pragma unroll
    for (int k = 0; k < TF_PER_LANE; ++k) {
      const int i = lane + 64 * k;
      if (i < TC_SAMPLE / 2) X[i] = p[k];
    }
    load(p, b + 2);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    f4 acc[2] = {f4{0.0f, 0.0f, 0.0f, 0.0f}, f4{0.0f, 0.0f, 0.0f, 0.0f}};
#pragma unroll
    for (int s = 0; s < TC_STEPS; ++s) {
      const uint16_t* row = Xh + (4 * s + kg) * TC_L + TC_S * rr;
      typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
      u16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = j < TC_K ? row[j] : (uint16_t)0;
      const bf8 a = __builtin_bit_cast(bf8, v);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bfr[s][nt], acc[nt], 0, 0, 0);
    }
    // C/D: column lane & 15, rows 4 (lane >> 4) + i
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int o = 16 * nt + (lane & 15);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int l = 4 * kg + i;
        if (l < TC_LOUT) y[((size_t)b * TC_LOUT + l) * TC_O + o] = bf16_bits(acc[nt][i] + bo[nt]);
      }
    }
    __builtin_amdgcn_wave_barrier();  // the next staging overwrites X after every lane's reads of it
  };
  for (int b = b0; b < b1; b += 2) {
    process(pa, b);
    if (b + 1 >= b1) break;
    process(pb, b + 1);
  }
}

// ---- weight gradient.  Workgroup g of TC_WG_BLOCKS: samples [b0, b1), staged one at a time into LDS (x: 3,102 bf16;
// gy: 14 x 32 bf16), the next sample's loads in flight.  Wave w owns column tiles w, w + 4, w + 8, w + 12 (< 13):
// A (32 x 16) = gy^T of the sample (rows o, k = output position l, rows 14, 15 zero), B (16 x 32) = the sample's
// unfolded inputs x[c, 3 l + t] for the tile's 32 (c, t) columns.
constexpr int TW_X = TC_SAMPLE / 2;       // 1,551 words
constexpr int TW_G = TC_LOUT * TC_O / 2;  // 224 words
constexpr int TW_LX = (TW_X + 255) / 256, TW_LG = (TW_G + 255) / 256;  // words per thread: 7, 1
__global__ __launch_bounds__(256) void k_conv1_wgrad_bf16(const uint16_t* __restrict__ x,
                                                          const uint16_t* __restrict__ gy, float* __restrict__ part,
                                                          int batch) {
  __shared__ uint32_t XS[2][TW_X + 1];
  __shared__ uint32_t GS[2][TW_G];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, h = lane >> 5, n = lane & 31;
  const int b0 = (int)((long long)blockIdx.x * batch / gridDim.x), b1 = (int)((long long)(blockIdx.x + 1) * batch / gridDim.x);
  const uint32_t* xw = reinterpret_cast<const uint32_t*>(x);
  const uint32_t* gw = reinterpret_cast<const uint32_t*>(gy);
  // three samples' loads in flight: register slots 0, 1, 2 hold samples b, b + 1, b + 2; a slot is refilled with sample
  // b + 3 (past the run: its last sample again, an L2 hit) as soon as it is staged, unconditionally, so the wait before
  // each staging counts only that slot's loads (one sample ahead: 2.5 TB/s, latency-bound)
  struct Slot {
    uint32_t x[TW_LX], g[TW_LG];
  };
  auto load = [&](Slot& sl, int bs) {
    const int bc = bs < b1 ? bs : b1 - 1;
    const uint32_t* sx = xw + (size_t)bc * TW_X;
    const uint32_t* sg = gw + (size_t)bc * TW_G;
#pragma unroll
    for (int k = 0; k < TW_LX; ++k) {
      const int i = t + 256 * k;
      sl.x[k] = sx[i < TW_X ? i : TW_X - 1];
    }
#pragma unroll
    for (int k = 0; k < TW_LG; ++k) {
      const int i = t + 256 * k;
      sl.g[k] = sg[i < TW_G ? i : TW_G - 1];
    }
  };
  // the tiles' (c, t) columns: col = 32 tile + n, c = col / 6, t = col % 6 (0 past the 396)
  constexpr int TPW = (TC_CT + 3) / 4;  // 4 tiles per wave at most
  int xoff[TPW];
  bool xcol[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int col = 32 * (wave + 4 * i) + n;
    xcol[i] = (wave + 4 * i) < TC_CT && col < TC_COLS;
    const int cc = xcol[i] ? col / TC_K : 0, tt = xcol[i] ? col % TC_K : 0;
    xoff[i] = cc * TC_L + tt;  // x[c, 3 l + t] = X[xoff + 3 l]
  }
  f16v acc[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[i][q] = 0.0f;
  float gbs = 0.0f;  // sum of this lane's gy values (o = n, positions 8 h .. 8 h + 7)
  Slot sl[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    load(sl[k], b0 + k);
    __builtin_amdgcn_sched_barrier(0);  // slot order = issue order
  }
  int buf = 0;
  auto sample = [&](Slot& cur, int b) {
#pragma unroll
    for (int k = 0; k < TW_LX; ++k) {
      const int i = t + 256 * k;
      if (i < TW_X) XS[buf][i] = cur.x[k];
    }
#pragma unroll
    for (int k = 0; k < TW_LG; ++k) {
      const int i = t + 256 * k;
      if (i < TW_G) GS[buf][i] = cur.g[k];
    }
    load(cur, b + 3);
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();  // staged (double-buffered: the sample before last's readers are done)
    const uint16_t* Xh = reinterpret_cast<const uint16_t*>(XS[buf]);
    const uint16_t* Gh = reinterpret_cast<const uint16_t*>(GS[buf]);
    typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
    // A: lane (o = n, h) holds gy[b, l = 8 h + j, o], zero for l >= 14
    u16x8 av;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int l = 8 * h + j;
      av[j] = l < TC_LOUT ? Gh[l * TC_O + n] : (uint16_t)0;
      gbs += bf16_float(av[j]);
    }
    const bf8 a = __builtin_bit_cast(bf8, av);
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      if (wave + 4 * i >= TC_CT) break;  // wave-uniform
      // B: lane (column n, h) holds x[c, 3 (8 h + j) + t], zero for positions >= 14 and past the 396 columns
      u16x8 bv;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int l = 8 * h + j;
        bv[j] = (l < TC_LOUT && xcol[i]) ? Xh[xoff[i] + TC_S * l] : (uint16_t)0;
      }
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, __builtin_bit_cast(bf8, bv), acc[i], 0, 0, 0);
    }
    buf ^= 1;
  };
  for (int b = b0; b < b1; b += 3) {
    sample(sl[0], b);
    if (b + 1 >= b1) break;
    sample(sl[1], b + 1);
    if (b + 2 >= b1) break;
    sample(sl[2], b + 2);
  }
  // the partial: [o][tile * 32 + n] (C/D: column n, row o = (q & 3) + 8 (q >> 2) + 4 h), then the 32 bias sums
  float* P = part + (size_t)blockIdx.x * TC_PART;
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    if (wave + 4 * i >= TC_CT) break;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int o = (q & 3) + 8 * (q >> 2) + 4 * h;
      P[(size_t)o * (TC_CT * 32) + 32 * (wave + 4 * i) + n] = acc[i][q];
    }
  }
  if (wave == 0) {
    gbs += __shfl_xor(gbs, 32);  // the two position halves of column o = n
    if (h == 0) P[TC_O * TC_CT * 32 + n] = gbs;
  }
}

// ---- the same weight gradient on fp32 operands (the fp32 update, the reference's precision: dh_ppo.py:155-182).  Each
// fp32 operand is split into three bf16 parts, v = v1 + v2 + v3 (v1 = bf16(v), v2 = bf16(v - v1), v3 = bf16(v - v1 - v2):
// 24+ significant bits, exact for normal fp32 values), and a product is formed from the six part products of order up
// to 2^-16 (a1 b1, a1 b2, a2 b1, a1 b3, a2 b2, a3 b1; the three dropped ones are below 2^-24 of |a b|), each exact in
// fp32 and accumulated by the MFMA in fp32: fp32-class sums (the tests hold them to 2e-6 of |gy|^T |x| against fp64).
// The staging, fragments and partials are k_conv1_wgrad_bf16's with fp32 rows in LDS (the parts are formed from them
// at fragment time); the bias sums the fp32 gy values.
struct Bf3 {
  bf8 p[3];
};
__device__ __forceinline__ void split_bf3(const float (&v)[8], Bf3& out) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 h1 = (__bf16)v[j];
    const float r1 = v[j] - (float)h1;
    const __bf16 h2 = (__bf16)r1;
    const float r2 = r1 - (float)h2;
    out.p[0][j] = h1;
    out.p[1][j] = h2;
    out.p[2][j] = (__bf16)r2;
  }
}
// acc += a b from the split operands: the smallest part products first
__device__ __forceinline__ f16v mfma_bf3(const Bf3& a, const Bf3& b, f16v acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[2], b.p[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[1], b.p[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[0], b.p[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[1], b.p[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[0], b.p[1], acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[0], b.p[0], acc, 0, 0, 0);
}
constexpr int TW32_X = TC_SAMPLE;          // 3,102 words
constexpr int TW32_G = TC_LOUT * TC_O;     // 448 words
constexpr int TW32_LX = (TW32_X + 255) / 256, TW32_LG = (TW32_G + 255) / 256;  // words per thread: 13, 2
__global__ __launch_bounds__(256) void k_conv1_wgrad_f32(const float* __restrict__ x, const float* __restrict__ gy,
                                                         float* __restrict__ part, int batch) {
  __shared__ float XS[2][TW32_X + 1];
  __shared__ float GS[2][TW32_G];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, h = lane >> 5, n = lane & 31;
  const int b0 = (int)((long long)blockIdx.x * batch / gridDim.x), b1 = (int)((long long)(blockIdx.x + 1) * batch / gridDim.x);
  // three samples' loads in flight, as k_conv1_wgrad_bf16
  struct Slot {
    float x[TW32_LX], g[TW32_LG];
  };
  auto load = [&](Slot& sl, int bs) {
    const int bc = bs < b1 ? bs : b1 - 1;
    const float* sx = x + (size_t)bc * TW32_X;
    const float* sg = gy + (size_t)bc * TW32_G;
#pragma unroll
    for (int k = 0; k < TW32_LX; ++k) {
      const int i = t + 256 * k;
      sl.x[k] = sx[i < TW32_X ? i : TW32_X - 1];
    }
#pragma unroll
    for (int k = 0; k < TW32_LG; ++k) {
      const int i = t + 256 * k;
      sl.g[k] = sg[i < TW32_G ? i : TW32_G - 1];
    }
  };
  constexpr int TPW = (TC_CT + 3) / 4;
  int xoff[TPW];
  bool xcol[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int col = 32 * (wave + 4 * i) + n;
    xcol[i] = (wave + 4 * i) < TC_CT && col < TC_COLS;
    const int cc = xcol[i] ? col / TC_K : 0, tt = xcol[i] ? col % TC_K : 0;
    xoff[i] = cc * TC_L + tt;
  }
  f16v acc[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[i][q] = 0.0f;
  float gbs = 0.0f;
  Slot sl[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    load(sl[k], b0 + k);
    __builtin_amdgcn_sched_barrier(0);
  }
  int buf = 0;
  auto sample = [&](Slot& cur, int b) {
#pragma unroll
    for (int k = 0; k < TW32_LX; ++k) {
      const int i = t + 256 * k;
      if (i < TW32_X) XS[buf][i] = cur.x[k];
    }
#pragma unroll
    for (int k = 0; k < TW32_LG; ++k) {
      const int i = t + 256 * k;
      if (i < TW32_G) GS[buf][i] = cur.g[k];
    }
    load(cur, b + 3);
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
    const float* X = XS[buf];
    const float* G = GS[buf];
    float av[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int l = 8 * h + j;
      av[j] = l < TC_LOUT ? G[l * TC_O + n] : 0.0f;
      gbs += av[j];
    }
    Bf3 a;
    split_bf3(av, a);
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      if (wave + 4 * i >= TC_CT) break;  // wave-uniform
      float bv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int l = 8 * h + j;
        bv[j] = (l < TC_LOUT && xcol[i]) ? X[xoff[i] + TC_S * l] : 0.0f;
      }
      Bf3 bb;
      split_bf3(bv, bb);
      acc[i] = mfma_bf3(a, bb, acc[i]);
    }
    buf ^= 1;
  };
  for (int b = b0; b < b1; b += 3) {
    sample(sl[0], b);
    if (b + 1 >= b1) break;
    sample(sl[1], b + 1);
    if (b + 2 >= b1) break;
    sample(sl[2], b + 2);
  }
  float* P = part + (size_t)blockIdx.x * TC_PART;
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    if (wave + 4 * i >= TC_CT) break;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int o = (q & 3) + 8 * (q >> 2) + 4 * h;
      P[(size_t)o * (TC_CT * 32) + 32 * (wave + 4 * i) + n] = acc[i][q];
    }
  }
  if (wave == 0) {
    gbs += __shfl_xor(gbs, 32);
    if (h == 0) P[TC_O * TC_CT * 32 + n] = gbs;
  }
}

// gW[o, c, t] (the (32, 66, 6) fp32 weight layout) and gb[o]: the partials summed in a fixed tree -- 16 groups per
// output (thread (g, o) sums partials g, g + 16, ... in order, eight loads in flight), then the 16 group sums in order
// (the one-thread-per-output chain of 512 dependent loads took 120 us, profiles/r05upd_*)
constexpr int TR_GROUPS = 16, TR_PER = 256 / TR_GROUPS;
__global__ __launch_bounds__(256) void k_conv1_wgrad_reduce(const float* __restrict__ part, int parts,
                                                            float* __restrict__ gw, float* __restrict__ gb) {
  __shared__ float red[256];
  const int g = threadIdx.x / TR_PER, o = threadIdx.x % TR_PER;
  const int e = blockIdx.x * TR_PER + o;
  const bool live = e < TC_O * TC_COLS + TC_O;
  int src = 0;
  if (live && e < TC_O * TC_COLS) {
    const int oc = e / TC_COLS, col = e % TC_COLS;
    src = oc * (TC_CT * 32) + col;
  } else if (live) {
    src = TC_O * TC_CT * 32 + (e - TC_O * TC_COLS);
  }
  float s = 0.0f;
  if (live) {
    int k = g;
    for (; k + 7 * TR_GROUPS < parts; k += 8 * TR_GROUPS) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(size_t)(k + u * TR_GROUPS) * TC_PART + src];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; k < parts; k += TR_GROUPS) s += part[(size_t)k * TC_PART + src];
  }
  red[threadIdx.x] = s;
  __syncthreads();
  if (g == 0 && live) {
    float sum = red[o];
#pragma unroll
    for (int q = 1; q < TR_GROUPS; ++q) sum += red[q * TR_PER + o];
    if (e < TC_O * TC_COLS) gw[e] = sum;
    else gb[e - TC_O * TC_COLS] = sum;
  }
}

// ---- column sums of a (rows, cols) gradient (the Linear bias gradients gy.sum(0) of the PPO update: 49,152 rows),
// fp32 accumulation in a fixed order: stage 1, block (column group of 64, chunk of CS_ROWS rows) -> partial; stage 2,
// the chunks summed in order
constexpr int CS_ROWS = 256;  // rows per stage-1 block: 49,152 rows -> 192 chunks (768 blocks at 256 columns)
template <typename T> __device__ __forceinline__ float cs_load(const T* p);
template <> __device__ __forceinline__ float cs_load<uint16_t>(const uint16_t* p) { return bf16_float(*p); }
template <> __device__ __forceinline__ float cs_load<float>(const float* p) { return *p; }
template <typename T>
__global__ __launch_bounds__(256) void k_colsum_part(const T* __restrict__ g, int rows, int cols, float* __restrict__ part) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), rg = threadIdx.x >> 6;
  const int r0 = blockIdx.y * CS_ROWS, r1 = r0 + CS_ROWS < rows ? r0 + CS_ROWS : rows;
  // rows rg, rg + 4, ... of the chunk: 8 independent loads and partial sums in flight, combined in a fixed order
  float s8[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
  if (c < cols) {
    for (int r = r0 + rg; r < r1; r += 32) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int rr = r + 4 * u;
        s8[u] += rr < r1 ? cs_load<T>(g + (size_t)rr * cols + c) : 0.0f;
      }
    }
  }
  const float s = ((s8[0] + s8[1]) + (s8[2] + s8[3])) + ((s8[4] + s8[5]) + (s8[6] + s8[7]));
  red[rg][threadIdx.x & 63] = s;
  __syncthreads();
  if (rg == 0 && c < cols)
    part[(size_t)blockIdx.y * cols + c] = ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
}
__global__ __launch_bounds__(256) void k_colsum_final(const float* __restrict__ part, int chunks, int cols,
                                                      float* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= cols) return;
  float s4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  int k = 0;
  for (; k + 4 <= chunks; k += 4)
#pragma unroll
    for (int u = 0; u < 4; ++u) s4[u] += part[(size_t)(k + u) * cols + c];
  for (; k < chunks; ++k) s4[0] += part[(size_t)k * cols + c];
  out[c] = (s4[0] + s4[1]) + (s4[2] + s4[3]);
}

// ---- the split-K weight gradient's partial products summed over the slices: out[i] = sum_s part[s][i], s in order
// (fp32; the PPO update's wgrad_splitk: 24 slices of M x N fp32 at 49,152 rows).  One thread per 4 consecutive
// outputs (float4 loads, 8 slices in flight); the sum runs s = 0, 1, ... exactly, so the result does not depend on the
// launch shape.
__global__ __launch_bounds__(256) void k_slice_sum4(const float4* __restrict__ part, int slices, int n4,
                                                    float4* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  float4 s = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  int k = 0;
  for (; k + 8 <= slices; k += 8) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = part[(size_t)(k + u) * n4 + i];
#pragma unroll
    for (int u = 0; u < 8; ++u) { s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w; }
  }
  for (; k < slices; ++k) {
    const float4 v = part[(size_t)k * n4 + i];
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  out[i] = s;
}
__global__ __launch_bounds__(256) void k_slice_sum1(const float* __restrict__ part, int slices, int n,
                                                    float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = 0.0f;
  for (int k = 0; k < slices; ++k) s += part[(size_t)k * n + i];
  out[i] = s;
}

// ---- the input gradient of an unfolded channels-last Conv1d (dh_policy._UnfoldRows: the history encoder's second conv
// as unfold + GEMM in the update): gx[b, l, c] = sum over taps t with l - t = stride p, 0 <= p < lout, of
// g[b, p, c, t] -- torch's unfold backward (a zero-filled scatter-add, 88 us per minibatch) as a gather, one
// workgroup per sample and one thread per (l, c), the taps in ascending order summed in fp32 and rounded once to the
// element type (bit-identical to the scatter-add when at most two taps meet, as at kernel 4 / stride 2)
template <typename E>
__global__ __launch_bounds__(256) void k_fold_rows(const E* __restrict__ g, E* __restrict__ gx, int batch, int length,
                                                   int channels, int kernel, int stride, int lout) {
  // one workgroup per sample (grid-stride), threads over the sample's (l, c) outputs: 32-bit index math inside a sample
  const int per = length * channels;
  for (int b = blockIdx.x; b < batch; b += gridDim.x) {
    const E* gb = g + (size_t)b * lout * channels * kernel;
    E* xb = gx + (size_t)b * per;
    for (int e = threadIdx.x; e < per; e += blockDim.x) {
      const int l = e / channels, c = e - l * channels;
      float s = 0.0f;
      for (int t = 0; t < kernel; ++t) {
        const int d = l - t;
        if (d < 0 || d % stride != 0 || d / stride >= lout) continue;
        const E v = gb[((d / stride) * channels + c) * kernel + t];
        if constexpr (sizeof(E) == 2) s += bf16_float(v);
        else s += __uint_as_float(v);
      }
      if constexpr (sizeof(E) == 2) xb[e] = bf16_bits(s);
      else xb[e] = __float_as_uint(s);
    }
  }
}

// the same for the update's shape, channels C / kernel K / stride S known at compile time: a thread owns one (l, c) of
// FR_SB consecutive samples and issues all their tap loads before any sum (the per-sample loop waited a full memory
// latency per sample: 74-97 us per minibatch)
constexpr int FR_SB = 8;
template <typename E, int C, int K, int S>
__global__ __launch_bounds__(256) void k_fold_rows_ks(const E* __restrict__ g, E* __restrict__ gx, int batch,
                                                      int length, int lout) {
  const int tid = blockIdx.x * 256 + threadIdx.x;
  const int c = tid % C, r = tid / C;
  const int l = r % length, b0 = (r / length) * FR_SB;
  if (b0 >= batch) return;
  E v[K][FR_SB];
#pragma unroll
  for (int t = 0; t < K; ++t) {
    const int d = l - t;
    const bool ok = d >= 0 && d % S == 0 && d / S < lout;
    const int p = ok ? d / S : 0;
#pragma unroll
    for (int u = 0; u < FR_SB; ++u) {
      const int b = b0 + u < batch ? b0 + u : batch - 1;
      v[t][u] = ok ? g[(((size_t)b * lout + p) * C + c) * K + t] : E(0);
    }
  }
#pragma unroll
  for (int u = 0; u < FR_SB; ++u) {
    if (b0 + u >= batch) break;
    float s = 0.0f;
#pragma unroll
    for (int t = 0; t < K; ++t) {
      const int d = l - t;
      if (d < 0 || d % S != 0 || d / S >= lout) continue;
      if constexpr (sizeof(E) == 2) s += bf16_float(v[t][u]);
      else s += __uint_as_float(v[t][u]);
    }
    E* xb = gx + ((size_t)(b0 + u) * length + l) * C + c;
    if constexpr (sizeof(E) == 2) *xb = bf16_bits(s);
    else *xb = __float_as_uint(s);
  }
}

bool tc_shape(int channels, int length, int out_channels, int kernel, int stride) {
  return channels == TC_C && length == TC_L && out_channels == TC_O && kernel == TC_K && stride == TC_S;
}

}  // namespace

extern "C" {

int t1policy_conv1_bf16_frag_bytes(void) { return TC_FRAG_BYTES; }

int t1policy_conv1_bf16_workspace_bytes(void) { return TC_WG_BLOCKS * TC_PART * 4; }

int t1policy_conv1_pack_bf16(const float* weight, void* frag, int channels, int out_channels, int kernel,
                             void* stream) {
  if (!weight || !frag) return -1;
  if (!tc_shape(channels, TC_L, out_channels, kernel, TC_S)) return 1;
  if ((reinterpret_cast<uintptr_t>(frag) & 15u) != 0) return -1;
  hipLaunchKernelGGL(k_conv1_pack_bf16, dim3((TC_STEPS * 2 * 64 + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     weight, reinterpret_cast<uint16_t*>(frag));
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int t1policy_conv1_forward_bf16(const void* x, const void* frag, const float* bias, void* y, int batch, int channels,
                                int length, int out_channels, int kernel, int stride, void* stream) {
  if (!x || !frag || !bias || !y || batch < 0) return -1;
  if (!tc_shape(channels, length, out_channels, kernel, stride)) return 1;
  if (batch == 0) return 0;
  if ((reinterpret_cast<uintptr_t>(x) & 3u) != 0 || (reinterpret_cast<uintptr_t>(frag) & 15u) != 0) return -1;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
      hipSuccess || cus <= 0) return -2;
  const long long need = ((long long)batch + TF_WAVES - 1) / TF_WAVES;
  const int grid = (int)(need < 2LL * cus ? need : 2LL * cus);
  hipLaunchKernelGGL(k_conv1_fwd_bf16, dim3(grid), dim3(64 * TF_WAVES), 0, (hipStream_t)stream,
                     reinterpret_cast<const uint16_t*>(x), reinterpret_cast<const bf8*>(frag), bias,
                     reinterpret_cast<uint16_t*>(y), batch);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int t1policy_conv1_wgrad_f32(const float* x, const float* gy, void* workspace, float* grad_weight, float* grad_bias,
                             int batch, int channels, int length, int out_channels, int kernel, int stride,
                             void* stream) {
  if (!x || !gy || !workspace || !grad_weight || !grad_bias || batch <= 0) return -1;
  if (!tc_shape(channels, length, out_channels, kernel, stride)) return 1;
  const int parts = batch < TC_WG_BLOCKS ? batch : TC_WG_BLOCKS;
  float* part = reinterpret_cast<float*>(workspace);
  hipLaunchKernelGGL(k_conv1_wgrad_f32, dim3(parts), dim3(256), 0, (hipStream_t)stream, x, gy, part, batch);
  hipLaunchKernelGGL(k_conv1_wgrad_reduce, dim3((TC_O * TC_COLS + TC_O + TR_PER - 1) / TR_PER), dim3(256), 0,
                     (hipStream_t)stream, part, parts, grad_weight, grad_bias);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int t1policy_conv1_wgrad_bf16(const void* x, const void* gy, void* workspace, float* grad_weight, float* grad_bias,
                              int batch, int channels, int length, int out_channels, int kernel, int stride,
                              void* stream) {
  if (!x || !gy || !workspace || !grad_weight || !grad_bias || batch <= 0) return -1;
  if (!tc_shape(channels, length, out_channels, kernel, stride)) return 1;
  if ((reinterpret_cast<uintptr_t>(x) & 3u) != 0 || (reinterpret_cast<uintptr_t>(gy) & 3u) != 0) return -1;
  const int parts = batch < TC_WG_BLOCKS ? batch : TC_WG_BLOCKS;
  float* part = reinterpret_cast<float*>(workspace);
  hipLaunchKernelGGL(k_conv1_wgrad_bf16, dim3(parts), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const uint16_t*>(x), reinterpret_cast<const uint16_t*>(gy), part, batch);
  hipLaunchKernelGGL(k_conv1_wgrad_reduce, dim3((TC_O * TC_COLS + TC_O + TR_PER - 1) / TR_PER), dim3(256), 0,
                     (hipStream_t)stream, part, parts, grad_weight, grad_bias);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int t1policy_colsum_workspace_bytes(int rows, int cols) {
  if (rows <= 0 || cols <= 0) return -1;
  return ((rows + CS_ROWS - 1) / CS_ROWS) * cols * 4;
}

int t1policy_colsum(const void* g, int elem_bytes, int rows, int cols, void* workspace, float* out, void* stream) {
  if (!g || !workspace || !out || rows <= 0 || cols <= 0) return -1;
  const int chunks = (rows + CS_ROWS - 1) / CS_ROWS;
  const dim3 grid((cols + 63) / 64, chunks);
  float* part = reinterpret_cast<float*>(workspace);
  if (elem_bytes == 2)
    hipLaunchKernelGGL(k_colsum_part<uint16_t>, grid, dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const uint16_t*>(g), rows, cols, part);
  else if (elem_bytes == 4)
    hipLaunchKernelGGL(k_colsum_part<float>, grid, dim3(256), 0, (hipStream_t)stream, reinterpret_cast<const float*>(g),
                       rows, cols, part);
  else
    return -1;
  hipLaunchKernelGGL(k_colsum_final, dim3((cols + 255) / 256), dim3(256), 0, (hipStream_t)stream, part, chunks, cols,
                     out);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int t1policy_fold_rows(const void* g, void* gx, int batch, int length, int channels, int kernel, int stride,
                       int elem_bytes, void* stream) {
  if (!g || !gx || batch < 0 || length <= 0 || channels <= 0 || kernel <= 0 || stride <= 0 || length < kernel)
    return -1;
  if (elem_bytes != 2 && elem_bytes != 4) return -1;
  if (batch == 0) return 0;
  const int lout = (length - kernel) / stride + 1;
  if ((long long)lout * channels * kernel >= (1LL << 31) || (long long)length * channels >= (1LL << 31)) return -1;
  const int grid = batch < 8192 ? batch : 8192;
  if (kernel == 4 && stride == 2 && channels == 32) {
    const long long threads = ((long long)(batch + FR_SB - 1) / FR_SB) * length * 32;
    const int fgrid = (int)((threads + 255) / 256);
    if (elem_bytes == 2)
      hipLaunchKernelGGL((k_fold_rows_ks<uint16_t, 32, 4, 2>), dim3(fgrid), dim3(256), 0, (hipStream_t)stream,
                         reinterpret_cast<const uint16_t*>(g), reinterpret_cast<uint16_t*>(gx), batch, length, lout);
    else
      hipLaunchKernelGGL((k_fold_rows_ks<uint32_t, 32, 4, 2>), dim3(fgrid), dim3(256), 0, (hipStream_t)stream,
                         reinterpret_cast<const uint32_t*>(g), reinterpret_cast<uint32_t*>(gx), batch, length, lout);
  } else if (elem_bytes == 2)
    hipLaunchKernelGGL(k_fold_rows<uint16_t>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const uint16_t*>(g), reinterpret_cast<uint16_t*>(gx), batch, length, channels,
                       kernel, stride, lout);
  else
    hipLaunchKernelGGL(k_fold_rows<uint32_t>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const uint32_t*>(g), reinterpret_cast<uint32_t*>(gx), batch, length, channels,
                       kernel, stride, lout);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int t1policy_slice_sum(const float* part, int slices, int n, float* out, void* stream) {
  if (!part || !out || slices <= 0 || n <= 0) return -1;
  if (n % 4 == 0 && (reinterpret_cast<uintptr_t>(part) & 15u) == 0 && (reinterpret_cast<uintptr_t>(out) & 15u) == 0) {
    const int n4 = n / 4;
    hipLaunchKernelGGL(k_slice_sum4, dim3((n4 + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const float4*>(part), slices, n4, reinterpret_cast<float4*>(out));
  } else {
    hipLaunchKernelGGL(k_slice_sum1, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, part, slices, n, out);
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
