// Direct Conv1d of the DH policy's long-history encoder, inference forward (include/t1policy.h).
//
// The reference's first history conv (actor_critic_dh.py:83-96): nn.Conv1d(66 frames -> 32, kernel 6, stride 3)
// over the 47 features of each frame.  y[b, l, o] = bias[o] + sum_{c, t} w[o, c, t] * x[b, c, S*l + t], written
// channels-last (B, Lout, O), the layout conv1d_as_gemm returns.
//
// One lane per output position (b, l) and group of 8 output channels: the weights are the same for every lane,
// so they are read with wave-uniform addresses (scalar loads, used as SGPR operands of the FMAs; the caller passes
// them tap-major, wt[c][t][o], so each (c, t) is O contiguous floats) and the only vector loads are the lane's own
// K inputs per channel.  That replaces the unfolded-row copy
// (B * Lout * C * K floats) plus a GEMM over it with one pass over x.  fp32 throughout; the sum runs over (c, t) in
// order, so the result equals the GEMM's up to fp32 summation order.
#include <hip/hip_runtime.h>

namespace {

template <int C, int L, int O, int K, int S, int OPL>
__global__ __launch_bounds__(256) void k_conv1d_direct(const float* __restrict__ x, const float* __restrict__ wt,
                                                       const float* __restrict__ bias, float* __restrict__ y,
                                                       int positions) {
  // blockIdx.y picks OPL of the O output channels (uniform per wave: the weights stay scalar loads); 4x the waves of
  // one lane per position with all O outputs, so the loads of one wave hide behind the FMAs of others
  constexpr int LOUT = (L - K) / S + 1;
  const int g = blockIdx.x * blockDim.x + threadIdx.x;  // output position b * LOUT + l
  if (g >= positions) return;
  const int o0 = blockIdx.y * OPL;
  const int b = g / LOUT, l = g - b * LOUT;
  const float* xp = x + (size_t)b * (C * L) + S * l;
  const float* wp = wt + o0;
  float acc[OPL];
#pragma unroll
  for (int o = 0; o < OPL; ++o) acc[o] = bias[o0 + o];
#pragma unroll 2
  for (int c = 0; c < C; ++c) {
    float xv[K];
#pragma unroll
    for (int t = 0; t < K; ++t) xv[t] = xp[c * L + t];
#pragma unroll
    for (int t = 0; t < K; ++t) {
#pragma unroll
      for (int o = 0; o < OPL; ++o) acc[o] = fmaf(wp[(c * K + t) * O + o], xv[t], acc[o]);
    }
  }
  float4* yp = reinterpret_cast<float4*>(y + (size_t)g * O + o0);
#pragma unroll
  for (int q = 0; q < OPL / 4; ++q) yp[q] = make_float4(acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]);
}

}  // namespace

extern "C" {

// Returns 0 on success, 1 if the shape has no compiled instance (the caller keeps its GEMM path), -1 on bad
// arguments, -2 on a launch error.
int t1policy_conv1d_forward(const float* x, const float* wt, const float* bias, float* y, int batch, int channels,
                            int length, int out_channels, int kernel, int stride, void* stream) {
  if (!x || !wt || !bias || !y || batch < 0) return -1;
  if (batch == 0) return 0;
  if (!(channels == 66 && length == 47 && out_channels == 32 && kernel == 6 && stride == 3)) return 1;
  constexpr int LOUT = (47 - 6) / 3 + 1;
  const long long positions = (long long)batch * LOUT;
  if (positions > 0x7fffffffLL) return -1;
  const int block = 256;
  const int grid = (int)((positions + block - 1) / block);
  constexpr int OPL = 8;
  hipLaunchKernelGGL((k_conv1d_direct<66, 47, 32, 6, 3, OPL>), dim3(grid, 32 / OPL), dim3(block), 0, (hipStream_t)stream, x, wt,
                     bias, y, (int)positions);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
