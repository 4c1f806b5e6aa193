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
// channels, 17 steps cover the 66 (2 zero channels).  Each workgroup builds the split weight fragments in LDS once;
// each wave stages one sample (12.4 KB, coalesced) into its own LDS rows while the next sample's loads are in flight.
#include <hip/hip_runtime.h>

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

// The PPO minibatch's actor observations rebuilt from the frame-history rollout storage (algo/rollout.py
// _HistoryRows): row m is the window of frames k .. k + F - 1 of env n's sequence seq[n] ((F + T - 1) frames of `frame`
// values, k = idx[m] / N, n = idx[m] % N), with the frames older than the env's latest reset at or before step k
// (time < first[k, n], time = k - F + 1 + j for window frame j) zeroed -- a prefix of the window.  One wave per row;
// 16-bit (bf16 / fp16 storage) or 32-bit elements copied as raw bits.
template <typename E>
__global__ __launch_bounds__(256) void k_history_rows(const E* __restrict__ seq, const int64_t* __restrict__ first,
                                                      const int64_t* __restrict__ idx, E* __restrict__ out, int rows,
                                                      int N, int T, int frames, int frame) {
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= rows) return;
  const int lane = threadIdx.x & 63;
  const int64_t g = idx[m];
  const int k = (int)(g / N), n = (int)(g % N);
  const int64_t f = first[(int64_t)k * N + n];
  const int64_t t0 = (int64_t)k - frames + 1;  // time of window frame 0
  const int64_t z = f - t0;
  const int zero_frames = z <= 0 ? 0 : (z >= frames ? frames : (int)z);
  const int len = frames * frame, zlen = zero_frames * frame;
  const E* src = seq + ((int64_t)n * (frames + T - 1) + k) * frame;
  E* dst = out + (int64_t)m * len;
  for (int i = lane; i < len; i += 64) dst[i] = i < zlen ? E(0) : src[i];
}

}  // namespace

extern "C" {

int t1policy_history_rows(const void* seq, const int64_t* first, const int64_t* idx, void* out, int rows, int num_envs,
                          int steps, int frames, int frame, int elem_bytes, void* stream) {
  if (!seq || !first || !idx || !out || rows < 0 || num_envs <= 0 || steps <= 0 || frames <= 0 || frame <= 0) return -1;
  if (rows == 0) return 0;
  const dim3 grid((rows + 3) / 4), block(256);
  if (elem_bytes == 2)
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

}  // extern "C"
