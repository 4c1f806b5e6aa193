/* t1policy.h -- C-ABI of the DH policy's HIP kernels (libt1env_hip.so, gfx950).
 *
 * Not an Isaac Gym replacement: the rollout-side policy forward that the reference
 * runs as torch nn.Conv1d (humanoid/algo/ppo/actor_critic_dh.py:83-96, the long-history encoder's first
 * Conv1d(66 -> 32, kernel 6, stride 3) over the 47 features of each of the 66 history frames).
 *
 * Plain device pointers, fp32, `stream` is a hipStream_t (0 = the null stream).
 */
#ifndef T1POLICY_H
#define T1POLICY_H

#ifdef __cplusplus
extern "C" {
#endif

/* y[b, l, o] = bias[o] + sum_{c,t} w[o, c, t] * x[b, c, stride*l + t] for l < (length - kernel) / stride + 1.
 *   x    (batch, channels, length), contiguous
 *   wt   the Conv1d weight tap-major: wt[(c * kernel + t) * out_channels + o] = weight[o, c, t]
 *   bias (out_channels)
 *   y    (batch, Lout, out_channels), channels-last
 * Returns 0 on success, 1 if the shape has no compiled instance (only 66/47/32/6/3 is), -1 on bad arguments,
 * -2 on a launch error.  Replaces (inference only, no autograd) nn.Conv1d.forward at actor_critic_dh.py:83-96. */
int t1policy_conv1d_forward(const float* x, const float* wt, const float* bias, float* y, int batch, int channels,
                            int length, int out_channels, int kernel, int stride, void* stream);

#ifdef __cplusplus
}
#endif
#endif
