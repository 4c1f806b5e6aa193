// Conv1d of the DH policy's long-history encoder, inference forward (include/t1policy.h), on the matrix cores.
//
// The reference's first history conv (actor_critic_dh.py:83-96): nn.Conv1d(66 frames -> 32, kernel 6, stride 3)
// over the 47 features of each frame.  y[b, l, o] = bias[o] + sum_{c, t} w[o, c, t] * x[b, c, S*l + t], written
// channels-last (B, Lout, O), the layout conv1d_as_gemm returns.
//
// Per sample it is a (14 positions x 396) . (396 x 32) product: one 16-row MFMA tile (rows 14, 15 discarded) and two
// 16-column tiles, v_mfma_f32_16x16x32_f16.  fp32 accuracy from fp16 matrix cores by splitting both operands:
// v = hi + lo with hi = fp16(v) and lo = fp16((v - hi) * 2^11) (the residual scaled up, so it does not underflow fp16),
// and y = sum hi.hi + 2^-11 sum (hi.lo + lo.hi): three MFMAs per step, fp32 accumulation, the dropped lo.lo term and
// the residual's rounding are ~2^-22 of each product (the test bound is 1e-5, tests/test_gpu_policy_conv.py).  The
// fp32 VALU kernel this replaces ran 66 us at 8192 samples (compute-bound: 2.9 GFLOP at <= 157 TFLOP/s fp32); the
// split runs on the 2.5 PFLOP/s fp16 rate and is bound by the 101.6 MB read of the history instead.
//
// K order: 8 slots per channel (its 6 taps and 2 zeros), so a lane's A fragment (row = output position l, 8 slots of
// one channel) is the 6 contiguous inputs x[c][3l .. 3l+5] and needs no transposition; a K-step of 32 covers 4
// channels, 17 steps cover the 66 (2 zero channels).  k_conv1d_mfma (t1policy_conv1d_forward, tap-major weights):
// each workgroup builds the split weight fragments in LDS once; each wave stages one sample (12.4 KB, coalesced)
// into its own LDS rows while the next sample's loads are in flight.  The packed form (t1policy_conv1d_pack_weights +
// t1policy_conv1d_forward_packed) takes fragments split once per weight version: k_conv1d_pair (default) and
// k_conv1d_regs (A/B), below.
#include <hip/hip_runtime.h>

#include <cstdlib>

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int CV_C = 66, CV_L = 47, CV_O = 32, CV_K = 6, CV_S = 3, CV_LOUT = (CV_L - CV_K) / CV_S + 1;  // 14
constexpr int CV_STEPS = 17;            // K-steps of 32: 4 channels each
constexpr int CV_CPAD = 4 * CV_STEPS;   // 68 staged channel rows (66 + 2 zero rows), 47 inputs each, unpadded: the
                                        // sample's own layout, so staging is a straight copy
constexpr int CV_WAVES = 6;             // waves per workgroup (LDS: 69.6 KB of fragments + 6 x 12.8 KB of samples)
constexpr int CV_PER_LANE = (CV_C * CV_L / 2 + 63) / 64;  // float2 loads per lane per sample (1551 float2)
constexpr float CV_SPLIT = 2048.0f;
static_assert(CV_LOUT <= 16 && CV_O == 32, "one 16-row tile, two 16-column tiles");

struct ConvLds {
  h8 wf[CV_STEPS][2][2][64];               // [step][column tile][hi, lo][lane]
  uint32_t x[CV_WAVES][CV_CPAD * CV_L];   // each wave's staged sample, split: hi (low 16 bits) | lo (high 16 bits)
};

__device__ __forceinline__ void split8(const float (&v)[8], h8& hi, h8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const _Float16 h = (_Float16)v[j];
    hi[j] = h;
    lo[j] = (_Float16)((v[j] - (float)h) * CV_SPLIT);
  }
}

// one input split at staging (once per element, not once per use): fp16 hi | fp16 lo << 16
__device__ __forceinline__ uint32_t split_word(float v) {
  const _Float16 h = (_Float16)v;
  const _Float16 l = (_Float16)((v - (float)h) * CV_SPLIT);
  return (uint32_t)__builtin_bit_cast(uint16_t, h) | ((uint32_t)__builtin_bit_cast(uint16_t, l) << 16);
}

__global__ __launch_bounds__(64 * CV_WAVES) void k_conv1d_mfma(const float* __restrict__ x, const float* __restrict__ wt,
                                                               const float* __restrict__ bias, float* __restrict__ y,
                                                               int batch) {
  __shared__ ConvLds L;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // the split weight fragments: lane l of (step s, column tile nt) holds B[k = 8 (l >> 4) + j][col l & 15], i.e.
  // channel c = 4 s + (l >> 4), tap j (< 6, else 0), output o = 16 nt + (l & 15)
  for (int e = tid; e < CV_STEPS * 2 * 64; e += 64 * CV_WAVES) {
    const int s = e >> 7, nt = (e >> 6) & 1, l = e & 63;
    const int c = 4 * s + (l >> 4), o = 16 * nt + (l & 15);
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (c < CV_C && j < CV_K) ? wt[(c * CV_K + j) * CV_O + o] : 0.0f;
    h8 hi, lo;
    split8(v, hi, lo);
    L.wf[s][nt][0][l] = hi;
    L.wf[s][nt][1][l] = lo;
  }
  uint32_t* X = L.x[wave];
  for (int i = CV_C * CV_L + lane; i < CV_CPAD * CV_L; i += 64) X[i] = 0u;  // the 2 zero channels stay zero
  __syncthreads();

  const int r = lane & 15, kg = lane >> 4;
  const int rr = r < CV_LOUT ? r : CV_LOUT - 1;  // rows 14, 15 of the tile: a copy of row 13, never stored
  const int stride = gridDim.x * CV_WAVES;
  int b = blockIdx.x * CV_WAVES + wave;
  // two samples in flight per wave: each buffer is refilled with the sample two strides ahead as soon as it is staged
  float2 pa[CV_PER_LANE], pb[CV_PER_LANE];
  auto load = [&](float2 (&dst)[CV_PER_LANE], int bs) {
    const float2* src = reinterpret_cast<const float2*>(x + (size_t)bs * (CV_C * CV_L));
#pragma unroll
    for (int k = 0; k < CV_PER_LANE; ++k) {
      const int i = lane + 64 * k;
      dst[k] = i < CV_C * CV_L / 2 ? src[i] : make_float2(0.0f, 0.0f);
    }
  };
  auto process = [&](float2 (&cur)[CV_PER_LANE], int bc) {
    // stage this sample (8-byte stores); the wave's own LDS rows: in-order LDS, no barrier
#pragma unroll
    for (int k = 0; k < CV_PER_LANE; ++k) {
      const int i = lane + 64 * k;
      if (i < CV_C * CV_L / 2) reinterpret_cast<uint2*>(X)[i] = make_uint2(split_word(cur[k].x), split_word(cur[k].y));
    }
    if (bc + 2 * stride < batch) load(cur, bc + 2 * stride);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    f4 acc[2][2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) acc[nt][0] = acc[nt][1] = f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int s = 0; s < CV_STEPS; ++s) {
      const uint32_t* row = X + (4 * s + kg) * CV_L + CV_S * rr;
      uint32_t w[CV_K];
#pragma unroll
      for (int j = 0; j < CV_K; ++j) w[j] = row[j];
      // hi halves (low 16 bits) and lo halves (high 16 bits) of taps 0..5 packed pairwise; taps 6, 7 zero
      typedef uint32_t u4 __attribute__((ext_vector_type(4)));
      const u4 hv = {__builtin_amdgcn_perm(w[1], w[0], 0x05040100u), __builtin_amdgcn_perm(w[3], w[2], 0x05040100u),
                     __builtin_amdgcn_perm(w[5], w[4], 0x05040100u), 0u};
      const u4 lv = {__builtin_amdgcn_perm(w[1], w[0], 0x07060302u), __builtin_amdgcn_perm(w[3], w[2], 0x07060302u),
                     __builtin_amdgcn_perm(w[5], w[4], 0x07060302u), 0u};
      const h8 ah = __builtin_bit_cast(h8, hv), al = __builtin_bit_cast(h8, lv);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const h8 bh = L.wf[s][nt][0][lane], bl = L.wf[s][nt][1][lane];
        acc[nt][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc[nt][0], 0, 0, 0);
        acc[nt][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, acc[nt][1], 0, 0, 0);
        acc[nt][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc[nt][1], 0, 0, 0);
      }
    }
    // C/D: column lane & 15, rows 4 (lane >> 4) + i
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int o = 16 * nt + (lane & 15);
      const float bo = bias[o];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int l = 4 * kg + i;
        if (l < CV_LOUT) y[((size_t)bc * CV_LOUT + l) * CV_O + o] = acc[nt][0][i] + acc[nt][1][i] * (1.0f / CV_SPLIT) + bo;
      }
    }
    // the next staging overwrites X: every lane's reads of it precede those writes in the wave's LDS order
    __builtin_amdgcn_wave_barrier();
  };
  if (b < batch) load(pa, b);
  if (b + stride < batch) load(pb, b + stride);
  for (; b < batch; b += 2 * stride) {
    process(pa, b);
    if (b + stride < batch) process(pb, b + stride);
  }
}

// ---- the packed-weight form (t1policy_conv1d_pack_weights + t1policy_conv1d_forward_packed).
// The split weight fragments are built once per weight version by k_conv1d_pack (CV_FRAG_BYTES, [step][column tile]
// [hi, lo][lane] h8, the layout of ConvLds::wf) and each wave of k_conv1d_regs holds all 68 of them in registers (272
// VGPRs, most in AGPRs, which the MFMAs read directly): no fragment LDS traffic (69.6 KB per sample in k_conv1d_mfma)
// and no per-workgroup fragment build.  One wave per SIMD; each wave takes a contiguous run of batch / waves samples
// (8 at 8192 on 256 CUs: balanced, where k_conv1d_mfma's 6 waves per CU ran 5 or 6 samples each, two waves sharing
// a SIMD), with the next two samples' loads in flight while it splits and multiplies the current one.
constexpr int CV_FRAGS = CV_STEPS * 2 * 2;                       // 68 h8 per lane
constexpr int CV_FRAG_BYTES = CV_FRAGS * 64 * 16;               // 69,632
constexpr int CR_WAVES = 4;

__global__ __launch_bounds__(256) void k_conv1d_pack(const float* __restrict__ w, h8* __restrict__ frag) {
  // w: the Conv1d weight as torch holds it, (O, C, K) contiguous
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < CV_STEPS * 2 * 64; e += gridDim.x * blockDim.x) {
    const int s = e >> 7, nt = (e >> 6) & 1, l = e & 63;
    const int c = 4 * s + (l >> 4), o = 16 * nt + (l & 15);
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (c < CV_C && j < CV_K) ? w[(o * CV_C + c) * CV_K + j] : 0.0f;
    h8 hi, lo;
    split8(v, hi, lo);
    frag[((s * 2 + nt) * 2 + 0) * 64 + l] = hi;
    frag[((s * 2 + nt) * 2 + 1) * 64 + l] = lo;
  }
}

__global__ __launch_bounds__(64 * CR_WAVES) __attribute__((amdgpu_waves_per_eu(1, 1)))
void k_conv1d_regs(const float* __restrict__ x, const h8* __restrict__ frag, const float* __restrict__ bias,
                   float* __restrict__ y, int batch) {
  __shared__ uint32_t XS[CR_WAVES][CV_CPAD * CV_L];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = blockIdx.x * CR_WAVES + wave, nw = gridDim.x * CR_WAVES;
  const int b0 = (int)((long long)g * batch / nw), b1 = (int)((long long)(g + 1) * batch / nw);
  uint32_t* X = XS[wave];
  for (int i = CV_C * CV_L + lane; i < CV_CPAD * CV_L; i += 64) X[i] = 0u;  // the 2 zero channels stay zero
  // the sample loads: 8-byte loads (a sample is 12,408 B, 8-byte aligned), 25 per lane, nothing past the sample
  float2 pa[CV_PER_LANE], pb[CV_PER_LANE];
  // every load and store of the loop is unconditional (clamped indices), so the compiler's vmcnt bookkeeping stays
  // exact and its waits for the current sample leave the next one's loads in flight
  auto load = [&](float2 (&dst)[CV_PER_LANE], int bs) {
    const float2* src = reinterpret_cast<const float2*>(x + (size_t)(bs < b1 ? bs : b1 - 1) * (CV_C * CV_L));
#pragma unroll
    for (int k = 0; k < CV_PER_LANE; ++k) {
      const int i = lane + 64 * k;
      dst[k] = src[i < CV_C * CV_L / 2 ? i : CV_C * CV_L / 2 - 1];
    }
  };
  if (b0 < b1) load(pa, b0);
  if (b0 + 1 < b1) load(pb, b0 + 1);
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  h8 bf[CV_STEPS][2][2];
#pragma unroll
  for (int s = 0; s < CV_STEPS; ++s)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int hl = 0; hl < 2; ++hl) bf[s][nt][hl] = frag[((s * 2 + nt) * 2 + hl) * 64 + lane];
  const int r = lane & 15, kg = lane >> 4;
  const int rr = r < CV_LOUT ? r : CV_LOUT - 1;  // rows 14, 15 of the tile: a copy of row 13, never stored
  float bo[2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) bo[nt] = bias[16 * nt + (lane & 15)];
  // the fragments retired before the loop (an empty asm use of each): otherwise the compiler's wait for them (the
  // youngest loads at the loop entry) stays inside the loop as a vmcnt that also drains the next sample's loads
#pragma unroll
  for (int s = 0; s < CV_STEPS; ++s)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int hl = 0; hl < 2; ++hl) asm volatile("" ::"v"(bf[s][nt][hl]));
  asm volatile("" ::"v"(bo[0]), "v"(bo[1]));  // the bias too
  auto process = [&](float2 (&cur)[CV_PER_LANE], int bc) {
#pragma unroll
    for (int k = 0; k < CV_PER_LANE; ++k) {
      const int i = lane + 64 * k;
      if (i < CV_C * CV_L / 2) reinterpret_cast<uint2*>(X)[i] = make_uint2(split_word(cur[k].x), split_word(cur[k].y));
    }
    load(cur, bc + 2);  // past the run: the run's last sample again (an L2 hit), not a branch
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    f4 acc[2][2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) acc[nt][0] = acc[nt][1] = f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int s = 0; s < CV_STEPS; ++s) {
      const uint32_t* row = X + (4 * s + kg) * CV_L + CV_S * rr;
      uint32_t w[CV_K];
#pragma unroll
      for (int j = 0; j < CV_K; ++j) w[j] = row[j];
      const u4 hv = {__builtin_amdgcn_perm(w[1], w[0], 0x05040100u), __builtin_amdgcn_perm(w[3], w[2], 0x05040100u),
                     __builtin_amdgcn_perm(w[5], w[4], 0x05040100u), 0u};
      const u4 lv = {__builtin_amdgcn_perm(w[1], w[0], 0x07060302u), __builtin_amdgcn_perm(w[3], w[2], 0x07060302u),
                     __builtin_amdgcn_perm(w[5], w[4], 0x07060302u), 0u};
      const h8 ah = __builtin_bit_cast(h8, hv), al = __builtin_bit_cast(h8, lv);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        acc[nt][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bf[s][nt][0], acc[nt][0], 0, 0, 0);
        acc[nt][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bf[s][nt][1], acc[nt][1], 0, 0, 0);
        acc[nt][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bf[s][nt][0], acc[nt][1], 0, 0, 0);
      }
    }
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int o = 16 * nt + (lane & 15);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        // tile rows 14, 15 repeat row 13's inputs, so their results are row 13's bit for bit: stored there again
        const int l = 4 * kg + i < CV_LOUT ? 4 * kg + i : CV_LOUT - 1;
        y[((size_t)bc * CV_LOUT + l) * CV_O + o] = acc[nt][0][i] + acc[nt][1][i] * (1.0f / CV_SPLIT) + bo[nt];
      }
    }
    __builtin_amdgcn_wave_barrier();  // the next staging overwrites X after every lane's reads of it
  };
  for (int b = b0; b < b1; b += 2) {
    process(pa, b);
    if (b + 1 < b1) process(pb, b + 1);
  }
}

// k_conv1d_pair: a workgroup is a pair of waves sharing each staged sample, wave w computing the 16 outputs of column
// tile w: it holds only its tile's 34 fragments (136 VGPRs), so two waves fit a SIMD (<= 256 VGPRs) and latency hides
// behind the other pair on it.  Each wave loads and splits half of every sample; the staged sample is double-buffered,
// one barrier per sample.  4 pairs per CU, a contiguous run of batch / pairs samples each (8 at 8192 on 256 CUs).
constexpr int CP_PAIRS_PER_CU = 4;
constexpr int CP_HALF = (CV_C * CV_L / 2 + 1) / 2;                 // 776 float2 of a sample per wave
constexpr int CP_PER_LANE = (CP_HALF + 63) / 64;                   // 13
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2, 2)))
void k_conv1d_pair(const float* __restrict__ x, const h8* __restrict__ frag, const float* __restrict__ bias,
                   float* __restrict__ y, int batch) {
  __shared__ uint32_t XS[2][CV_CPAD * CV_L];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // column tile of this wave
  const int b0 = (int)((long long)blockIdx.x * batch / gridDim.x), b1 = (int)((long long)(blockIdx.x + 1) * batch / gridDim.x);
  for (int i = CV_C * CV_L + (int)threadIdx.x; i < CV_CPAD * CV_L; i += 128) { XS[0][i] = 0u; XS[1][i] = 0u; }
  const int h0 = w * CP_HALF, h1 = w == 0 ? CP_HALF : CV_C * CV_L / 2;  // this wave's float2 range of a sample
  float2 pa[CP_PER_LANE], pb[CP_PER_LANE];
  // unconditional, clamped loads (exact vmcnt bookkeeping; past the run: the run's last sample again, an L2 hit)
  auto load = [&](float2 (&dst)[CP_PER_LANE], int bs) {
    const float2* src = reinterpret_cast<const float2*>(x + (size_t)(bs < b1 ? bs : b1 - 1) * (CV_C * CV_L));
#pragma unroll
    for (int k = 0; k < CP_PER_LANE; ++k) {
      const int i = h0 + lane + 64 * k;
      dst[k] = src[i < h1 ? i : h1 - 1];
    }
  };
  if (b0 < b1) {
    load(pa, b0);
    load(pb, b0 + 1);
  }
  h8 bf[CV_STEPS][2];
#pragma unroll
  for (int s = 0; s < CV_STEPS; ++s)
#pragma unroll
    for (int hl = 0; hl < 2; ++hl) bf[s][hl] = frag[((s * 2 + w) * 2 + hl) * 64 + lane];
  const float bo = bias[16 * w + (lane & 15)];
  // the fragments and the bias retired before the loop (see k_conv1d_regs)
#pragma unroll
  for (int s = 0; s < CV_STEPS; ++s) asm volatile("" ::"v"(bf[s][0]), "v"(bf[s][1]));
  asm volatile("" ::"v"(bo));
  const int r = lane & 15, kg = lane >> 4;
  const int rr = r < CV_LOUT ? r : CV_LOUT - 1;
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  auto process = [&](float2 (&cur)[CP_PER_LANE], int bc, uint32_t* X) {
#pragma unroll
    for (int k = 0; k < CP_PER_LANE; ++k) {
      const int i = h0 + lane + 64 * k;
      if (i < h1) reinterpret_cast<uint2*>(X)[i] = make_uint2(split_word(cur[k].x), split_word(cur[k].y));
    }
    load(cur, bc + 2);
    __syncthreads();  // both halves staged (and, X being double-buffered, both waves done with the sample before last)
    f4 acc0 = f4{0.0f, 0.0f, 0.0f, 0.0f}, acc1 = f4{0.0f, 0.0f, 0.0f, 0.0f};
#ifdef T1_CONV_WHATIF_NO_MFMA  // timing-only what-if build: the staging, loads and stores without the K loop
    acc0[0] = __uint_as_float(X[lane]);
#else
#pragma unroll
    for (int s = 0; s < CV_STEPS; ++s) {
      const uint32_t* row = X + (4 * s + kg) * CV_L + CV_S * rr;
      uint32_t v[CV_K];
#pragma unroll
      for (int j = 0; j < CV_K; ++j) v[j] = row[j];
      const u4 hv = {__builtin_amdgcn_perm(v[1], v[0], 0x05040100u), __builtin_amdgcn_perm(v[3], v[2], 0x05040100u),
                     __builtin_amdgcn_perm(v[5], v[4], 0x05040100u), 0u};
      const u4 lv = {__builtin_amdgcn_perm(v[1], v[0], 0x07060302u), __builtin_amdgcn_perm(v[3], v[2], 0x07060302u),
                     __builtin_amdgcn_perm(v[5], v[4], 0x07060302u), 0u};
      const h8 ah = __builtin_bit_cast(h8, hv), al = __builtin_bit_cast(h8, lv);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bf[s][0], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bf[s][1], acc1, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bf[s][0], acc1, 0, 0, 0);
    }
#endif
    const int o = 16 * w + (lane & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int l = 4 * kg + i < CV_LOUT ? 4 * kg + i : CV_LOUT - 1;  // rows 14, 15 = row 13's result, bit for bit
      y[((size_t)bc * CV_LOUT + l) * CV_O + o] = acc0[i] + acc1[i] * (1.0f / CV_SPLIT) + bo;
    }
  };
  for (int b = b0; b < b1; b += 2) {
    process(pa, b, XS[0]);
    if (b + 1 < b1) process(pb, b + 1, XS[1]);
  }
}

// The PPO minibatch's actor observations rebuilt from the frame-history rollout storage (algo/rollout.py
// _HistoryRows): row m is the window of frames k .. k + F - 1 of env n's sequence seq[n] ((F + T - 1) frames of `frame`
// values, k = idx[m] / N, n = idx[m] % N), with the frames older than the env's latest reset at or before step k
// (time < first[k, n], time = k - F + 1 + j for window frame j) zeroed -- a prefix of the window.  One wave per row,
// copied as 32-bit words in bursts of 8 per lane (eight loads in flight before the stores; the one-element-per-lane
// loop waited a full memory latency per 128 B, 181 us per 49,152-row minibatch, profiles/r05upd_*).  16-bit elements
// with an even row length: the row's words realigned from the source's parity (one extra aligned word, a 16-bit
// shift; the source window of an odd offset reaches one element past its last, inside the same aligned word);
// otherwise one element per lane.
struct HrRow {
  int64_t src;  // element offset of the window in seq
  int zlen;     // zeroed leading elements
};
__device__ __forceinline__ HrRow hr_row(const int64_t* __restrict__ first, const int64_t* __restrict__ idx, int m, int N,
                                        int T, int frames, int frame) {
  const int64_t g = idx[m];
  const int k = (int)(g / N), n = (int)(g % N);
  const int64_t f = first[(int64_t)k * N + n];
  const int64_t z = f - ((int64_t)k - frames + 1);  // frames before the reset (window frame 0 at time k - F + 1)
  const int zero_frames = z <= 0 ? 0 : (z >= frames ? frames : (int)z);
  return HrRow{((int64_t)n * (frames + T - 1) + k) * frame, zero_frames * frame};
}

constexpr int HR_BURST = 8;

template <typename E>
__global__ __launch_bounds__(256) void k_history_rows(const E* __restrict__ seq, const int64_t* __restrict__ first,
                                                      const int64_t* __restrict__ idx, E* __restrict__ out, int rows,
                                                      int N, int T, int frames, int frame) {
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= rows) return;
  const int lane = threadIdx.x & 63;
  const HrRow r = hr_row(first, idx, m, N, T, frames, frame);
  const int len = frames * frame;
  const E* src = seq + r.src;
  E* dst = out + (int64_t)m * len;
  for (int i0 = 0; i0 < len; i0 += 64 * HR_BURST) {
    E v[HR_BURST];
#pragma unroll
    for (int u = 0; u < HR_BURST; ++u) {
      const int i = i0 + 64 * u + lane;
      v[u] = src[i < len ? i : len - 1];
    }
#pragma unroll
    for (int u = 0; u < HR_BURST; ++u) {
      const int i = i0 + 64 * u + lane;
      if (i < len) dst[i] = i < r.zlen ? E(0) : v[u];
    }
  }
}

// 16-bit elements, even row length (dst rows start on 4-byte boundaries): 32-bit words
__global__ __launch_bounds__(256) void k_history_rows_w16(const uint16_t* __restrict__ seq,
                                                          const int64_t* __restrict__ first,
                                                          const int64_t* __restrict__ idx, uint16_t* __restrict__ out,
                                                          int rows, int N, int T, int frames, int frame) {
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= rows) return;
  const int lane = threadIdx.x & 63;
  const HrRow r = hr_row(first, idx, m, N, T, frames, frame);
  const int nw = frames * frame / 2;
  const bool odd = (r.src & 1) != 0;  // wave-uniform
  const uint32_t* sw = reinterpret_cast<const uint32_t*>(seq) + (r.src >> 1);  // the word holding the first element
  uint32_t* dw = reinterpret_cast<uint32_t*>(out + (int64_t)m * 2 * nw);
  // seq holds N * (frames + T - 1) * frame elements: with an odd count its last word is half outside the buffer.  An odd
  // window ending on the last element reads that element from the word past it (hi): clamp the word to the last whole one
  // and take the element by a 16-bit load instead
  const int64_t tot = (int64_t)N * (frames + T - 1) * frame;
  const int64_t hi_max = tot / 2 - 1 - (r.src >> 1);  // the last whole word, relative to sw
  for (int j0 = 0; j0 < nw; j0 += 64 * HR_BURST) {
    uint32_t lo[HR_BURST], hi[HR_BURST];
#pragma unroll
    for (int u = 0; u < HR_BURST; ++u) {
      int j = j0 + 64 * u + lane;
      j = j < nw ? j : nw - 1;
      lo[u] = sw[j];
      const int64_t jh = odd ? j + 1 : j;
      hi[u] = sw[jh < hi_max ? jh : hi_max];
    }
#pragma unroll
    for (int u = 0; u < HR_BURST; ++u) {
      const int j = j0 + 64 * u + lane;
      if (j >= nw) continue;
      if (odd && j + 1 > hi_max) hi[u] = seq[r.src + 2 * (int64_t)j + 1];  // the buffer's last element (rare)
      uint32_t w = odd ? (lo[u] >> 16) | (hi[u] << 16) : lo[u];
      if (2 * j + 1 < r.zlen) w = 0u;
      else if (2 * j < r.zlen) w &= 0xffff0000u;
      dw[j] = w;
    }
  }
}

// The PPO minibatch's per-transition fields gathered by one launch (rollout.py minibatch_source: critic observations,
// actions, values, advantages, returns, log-probs, means, sigmas -- eight torch index kernels before): field f's row
// m = src_f[idx[m]] (width_f 32-bit words).  One thread per (row, word) of the fields' concatenated row, so every field
// width is copied by whole waves.
constexpr int GR_MAX = 12;
struct GrFields {
  const uint32_t* src[GR_MAX];
  uint32_t* dst[GR_MAX];
  int width[GR_MAX];
  int off[GR_MAX + 1];  // prefix sums of the widths
  int n;
};
__global__ __launch_bounds__(256) void k_gather_rows(GrFields F, const int64_t* __restrict__ idx, int rows) {
  const int total = F.off[F.n];
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)rows * total) return;
  const int m = (int)(t / total), k = (int)(t - (long long)m * total);
  int f = 0;
#pragma unroll
  for (int q = 1; q < GR_MAX; ++q) f += (q < F.n && k >= F.off[q]) ? 1 : 0;
  const int w = F.width[f], c = k - F.off[f];
  F.dst[f][(size_t)m * w + c] = F.src[f][(size_t)idx[m] * w + c];
}

}  // namespace

extern "C" {

int t1policy_gather_rows(const void* const* srcs, void* const* dsts, const int* widths, int nfields,
                         const int64_t* idx, int rows, void* stream) {
  if (!srcs || !dsts || !widths || !idx || nfields <= 0 || nfields > GR_MAX || rows < 0) return -1;
  if (rows == 0) return 0;
  GrFields F{};
  F.off[0] = 0;
  for (int f = 0; f < nfields; ++f) {
    if (!srcs[f] || !dsts[f] || widths[f] <= 0 || widths[f] > (1 << 20)) return -1;
    F.src[f] = reinterpret_cast<const uint32_t*>(srcs[f]);
    F.dst[f] = reinterpret_cast<uint32_t*>(dsts[f]);
    F.width[f] = widths[f];
    F.off[f + 1] = F.off[f] + widths[f];
  }
  F.n = nfields;
  const long long threads = (long long)rows * F.off[nfields];
  hipLaunchKernelGGL(k_gather_rows, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, (hipStream_t)stream, F, idx,
                     rows);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}


int t1policy_history_rows(const void* seq, const int64_t* first, const int64_t* idx, void* out, int rows, int num_envs,
                          int steps, int frames, int frame, int elem_bytes, void* stream) {
  if (!seq || !first || !idx || !out || rows < 0 || num_envs <= 0 || steps <= 0 || frames <= 0 || frame <= 0) return -1;
  if (rows == 0) return 0;
  const dim3 grid((rows + 3) / 4), block(256);
  if (elem_bytes == 2 && (frames * frame) % 2 == 0 && (reinterpret_cast<uintptr_t>(seq) & 3u) == 0 &&
      (reinterpret_cast<uintptr_t>(out) & 3u) == 0)
    hipLaunchKernelGGL(k_history_rows_w16, grid, block, 0, (hipStream_t)stream, (const uint16_t*)seq, first, idx,
                       (uint16_t*)out, rows, num_envs, steps, frames, frame);
  else if (elem_bytes == 2)
    hipLaunchKernelGGL(k_history_rows<uint16_t>, grid, block, 0, (hipStream_t)stream, (const uint16_t*)seq, first, idx,
                       (uint16_t*)out, rows, num_envs, steps, frames, frame);
  else if (elem_bytes == 4)
    hipLaunchKernelGGL(k_history_rows<uint32_t>, grid, block, 0, (hipStream_t)stream, (const uint32_t*)seq, first, idx,
                       (uint32_t*)out, rows, num_envs, steps, frames, frame);
  else
    return -1;
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Returns 0 on success, 1 if the shape has no compiled instance (the caller keeps its GEMM path), -1 on bad
// arguments, -2 on a launch error.
int t1policy_conv1d_forward(const float* x, const float* wt, const float* bias, float* y, int batch, int channels,
                            int length, int out_channels, int kernel, int stride, void* stream) {
  if (!x || !wt || !bias || !y || batch < 0) return -1;
  if (batch == 0) return 0;
  if (!(channels == CV_C && length == CV_L && out_channels == CV_O && kernel == CV_K && stride == CV_S)) return 1;
  if ((reinterpret_cast<uintptr_t>(x) & 7u) != 0) return -1;  // float2 sample loads
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -2;
  static int cu_count[64];  // per device, queried once
  int cus = __atomic_load_n(&cu_count[dev], __ATOMIC_RELAXED);
  if (cus <= 0) {
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) return -2;
    __atomic_store_n(&cu_count[dev], cus, __ATOMIC_RELAXED);
  }
  // one workgroup per CU (its LDS), never more workgroups than the samples need
  const long long need = ((long long)batch + CV_WAVES - 1) / CV_WAVES;
  const int grid = (int)(need < cus ? need : cus);
  hipLaunchKernelGGL(k_conv1d_mfma, dim3(grid), dim3(64 * CV_WAVES), 0, (hipStream_t)stream, x, wt, bias, y, batch);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int t1policy_conv1d_frag_bytes(void) { return CV_FRAG_BYTES; }

int t1policy_conv1d_pack_weights(const float* w, void* frag, int channels, int out_channels, int kernel,
                                 void* stream) {
  if (!w || !frag) return -1;
  if (!(channels == CV_C && out_channels == CV_O && kernel == CV_K)) return 1;
  if ((reinterpret_cast<uintptr_t>(frag) & 15u) != 0) return -1;
  hipLaunchKernelGGL(k_conv1d_pack, dim3(CV_STEPS * 2 * 64 / 256 + 1), dim3(256), 0, (hipStream_t)stream, w,
                     reinterpret_cast<h8*>(frag));
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int t1policy_conv1d_forward_packed(const float* x, const void* frag, const float* bias, float* y, int batch,
                                   int channels, int length, int out_channels, int kernel, int stride, void* stream) {
  if (!x || !frag || !bias || !y || batch < 0) return -1;
  if (batch == 0) return 0;
  if (!(channels == CV_C && length == CV_L && out_channels == CV_O && kernel == CV_K && stride == CV_S)) return 1;
  if ((reinterpret_cast<uintptr_t>(x) & 15u) != 0 || (reinterpret_cast<uintptr_t>(frag) & 15u) != 0) return -1;
  if ((long long)batch * (CV_C * CV_L * 4) > 0x7fffffffLL) return -1;  // 32-bit buffer offsets
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -2;
  static int cu_count[64];
  int cus = __atomic_load_n(&cu_count[dev], __ATOMIC_RELAXED);
  if (cus <= 0) {
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) return -2;
    __atomic_store_n(&cu_count[dev], cus, __ATOMIC_RELAXED);
  }
  // k_conv1d_pair (default): CP_PAIRS_PER_CU two-wave workgroups per CU; T1POLICY_CONV=regs: k_conv1d_regs, one
  // 4-wave workgroup per CU (A/B).  No workgroup without a sample.
  const char* kv = getenv("T1POLICY_CONV");
  if (kv && kv[0] == 'r') {
    const long long need = ((long long)batch + CR_WAVES - 1) / CR_WAVES;
    const int grid = (int)(need < cus ? need : cus);
    hipLaunchKernelGGL(k_conv1d_regs, dim3(grid), dim3(64 * CR_WAVES), 0, (hipStream_t)stream, x,
                       reinterpret_cast<const h8*>(frag), bias, y, batch);
  } else {
    const char* pv = getenv("T1POLICY_CONV_PAIRS");  // pairs per CU (A/B; 1-6 fit the LDS)
    const int pairs = pv && atoi(pv) >= 1 && atoi(pv) <= 6 ? atoi(pv) : CP_PAIRS_PER_CU;
    const long long slots = (long long)cus * pairs;
    const int grid = (int)(batch < slots ? batch : slots);
    hipLaunchKernelGGL(k_conv1d_pair, dim3(grid), dim3(128), 0, (hipStream_t)stream, x,
                       reinterpret_cast<const h8*>(frag), bias, y, batch);
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
