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

#include <stdint.h>

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

/* The same convolution with the weight prepared once per weight version (the rollout's act(): the weights change
 * only at the PPO update).  pack_weights builds the kernel's split fp16 fragments of weight (out_channels, channels,
 * kernel) -- the layout torch's nn.Conv1d holds -- into frag (frag_bytes() bytes, 16-byte aligned, caller-owned
 * device memory); forward_packed then reads frag instead of a tap-major weight.  x and frag 16-byte aligned,
 * batch * channels * length * 4 < 2^31.  Same results as t1policy_conv1d_forward up to fp32 summation order
 * (both within 1e-5 * (1 + |y|) of an fp64 conv); same return codes. */
int t1policy_conv1d_frag_bytes(void);
int t1policy_conv1d_pack_weights(const float* weight, void* frag, int channels, int out_channels, int kernel,
                                 void* stream);
int t1policy_conv1d_forward_packed(const float* x, const void* frag, const float* bias, float* y, int batch,
                                   int channels, int length, int out_channels, int kernel, int stride, void* stream);

/* The rest of the rollout's act() after the first conv, one fused kernel (t1policy_heads.hip): the history tail
 * (conv2 + ReLU, flatten, 96 -> 128 ELU -> 64), the state estimator (235 -> 256 -> 128 -> 64 -> 3, ELU), the actor
 * ([short | estimate | code] 302 -> 512 -> 256 -> 128 -> 12, ELU), the critic (219 -> 768 -> 256 -> 128 -> 1, ELU),
 * and the Normal sample of DHPPO._act_body.  Replaces ActorCriticDH.act / evaluate / get_actions_log_prob
 * (actor_critic_dh.py:45-111,163-188; the torch restatement ti5_isaacgym_amd/algo/dh_policy.py) for inference.
 *
 *   params  host array of 31 device pointers, fp32, contiguous: (weight, bias) of the 15 layers in the order
 *           conv2, history fc1, fc2, estimator 1..4, actor 1..4, critic 1..4, then the 12 action stds
 *   dims    host array of 30 ints, (out, in) per layer (conv2: 16, 32 * 4): checked against the compiled shapes
 *   frag    heads_frag_bytes() bytes of device memory (16-byte aligned) that heads_pack fills from params (split
 *           fp16 fragments) and heads_forward reads; pack again after any weight change
 *   y1      the first conv's output (batch, 14, 32) channels-last (t1policy_conv1d_forward_packed), before its ReLU
 *   obs     (batch, obs_cols) actor observations, the short history = the last 235 columns
 *   critic_obs (batch, 219); eps (batch, 12) standard-normal draws
 *   out     mean, actions = mean + std eps, sigma (batch, 12); logp (batch) = sum of the Normal log-densities of
 *           actions; value (batch)
 * fp32 results within ~1e-6 relative of an fp64 forward (split fp16 matrix cores, fp32 accumulation).  Returns 0,
 * 1 for shapes without a compiled instance, -1 on bad arguments, -2 on a launch error. */
int t1policy_heads_frag_bytes(void);
int t1policy_heads_pack(const uint64_t* params, const int* dims, void* frag, void* stream);
int t1policy_heads_forward(const uint64_t* params, const int* dims, const void* frag, const float* y1,
                           const float* obs, int obs_cols, const float* critic_obs, int critic_cols, const float* eps,
                           float* mean, float* actions, float* sigma, float* logp, float* value, int batch,
                           void* stream);

/* The same first conv in the PPO update under the opt-in bf16 update (t1policy_train.hip), forward and weight
 * gradient on bf16 inputs without the unfolded copy (the autograd path dh_policy.conv1d_as_gemm unfolds 545 MB per
 * minibatch).  Shapes as t1policy_conv1d_forward (only 66/47/32/6/3 compiled; 1 otherwise).
 *   pack_bf16      weight (out_channels, channels, kernel) fp32 -> frag (frag_bytes(), 16-byte aligned): bf16 (round
 *                  to nearest even, as torch's .to(torch.bfloat16)) fragments
 *   forward_bf16   x (batch, channels, length) bf16 -> y (batch, Lout, out_channels) bf16 = bf16(fp32 sum of the bf16
 *                  products + bf16(bias)), autocast's addmm arithmetic; x 4-byte aligned
 *   wgrad_bf16     grad_weight (out_channels, channels, kernel) fp32 = sum_{b,l} gy[b,l,o] x[b,c,stride l + t],
 *                  grad_bias (out_channels) fp32 = sum gy, from gy (batch, Lout, out_channels) bf16; workspace of
 *                  workspace_bytes() device bytes; the per-workgroup partials are summed in a fixed order
 *                  (deterministic)
 * Replaces the training-time nn.Conv1d forward / weight gradient at actor_critic_dh.py:83-96. */
int t1policy_conv1_bf16_frag_bytes(void);
int t1policy_conv1_bf16_workspace_bytes(void);
int t1policy_conv1_pack_bf16(const float* weight, void* frag, int channels, int out_channels, int kernel, void* stream);
int t1policy_conv1_forward_bf16(const void* x, const void* frag, const float* bias, void* y, int batch, int channels,
                                int length, int out_channels, int kernel, int stride, void* stream);
int t1policy_conv1_wgrad_bf16(const void* x, const void* gy, void* workspace, float* grad_weight, float* grad_bias,
                              int batch, int channels, int length, int out_channels, int kernel, int stride,
                              void* stream);
/* The same weight gradient on fp32 x (batch, channels, length) and gy (batch, Lout, out_channels) -- the fp32 update,
 * the reference's precision (dh_ppo.py:155-182) -- on the matrix cores: each fp32 operand split into three bf16 parts,
 * the six part products down to 2^-16 of each product formed by v_mfma_f32_32x32x16_bf16 and summed in fp32
 * (fp32-class: within 2e-6 of |gy|^T |x| of the fp64 sum in tests/test_gpu_conv1_train.py); grad_bias the fp32 sum of
 * gy.  workspace: t1policy_conv1_bf16_workspace_bytes() device bytes; the same fixed-order partial sums
 * (deterministic).  The forward of the fp32 update is t1policy_conv1d_forward_packed (fp32-accurate, above). */
int t1policy_conv1_wgrad_f32(const float* x, const float* gy, void* workspace, float* grad_weight, float* grad_bias,
                             int batch, int channels, int length, int out_channels, int kernel, int stride,
                             void* stream);

/* Column sums of a (rows, cols) row-major gradient, bf16 (elem_bytes 2) or fp32 (4): out[c] = sum_r g[r, c] in fp32,
 * in a fixed order (workspace of colsum_workspace_bytes(rows, cols) device bytes): the PPO update's Linear bias
 * gradients (gy.sum(0) in dh_policy._LinearSplitK; torch's dim-0 sum ran 8-32 us per call at 49,152 rows).
 * Returns 0, -1 on bad arguments, -2 on a launch error. */
int t1policy_colsum_workspace_bytes(int rows, int cols);
int t1policy_colsum(const void* g, int elem_bytes, int rows, int cols, void* workspace, float* out, void* stream);
/* The split-K weight gradient's reduction (dh_policy.wgrad_splitk; replaces torch's part.sum(0) after the batched GEMM,
 * the reduction inside dh_ppo.py:180's loss.backward() for every Linear weight, humanoid/algo/ppo/dh_ppo.py:112-205):
 * out[i] = sum over s = 0 .. slices-1, in that order, of part[s * n + i] (fp32).  Returns 0, -1 bad arguments, -2 launch
 * error. */
int t1policy_slice_sum(const float* part, int slices, int n, float* out, void* stream);

/* The PPO minibatch's per-transition fields in one launch (the reference's generator indexes each buffer,
 * rollout_storage.py:153-173; ti5_isaacgym_amd/algo/rollout.py minibatch_source): for f < nfields (<= 12) and
 * m < rows, dsts[f][m, :] = srcs[f][idx[m], :], rows of widths[f] 32-bit words, row-major.  Returns 0, -1 on bad
 * arguments, -2 on a launch error. */
int t1policy_gather_rows(const void* const* srcs, void* const* dsts, const int* widths, int nfields,
                         const int64_t* idx, int rows, void* stream);

/* The input gradient of a channels-last Conv1d run as unfold + GEMM (the history encoder's second conv in the PPO
 * update, actor_critic_dh.py:83-96; replaces torch's unfold backward inside dh_ppo.py:180's loss.backward()):
 *   gx[b, l, c] = sum over taps t (ascending) with l - t = stride * p, 0 <= p < lout, of g[b, p, c, t]
 * g: (batch, lout, channels, kernel) row-major, gx: (batch, length, channels), lout = (length - kernel) / stride + 1;
 * elem_bytes 2 (bf16) or 4 (fp32), summed in fp32 and rounded once.  Returns 0, -1 on bad arguments, -2 on a launch
 * error. */
int t1policy_fold_rows(const void* g, void* gx, int batch, int length, int channels, int kernel, int stride,
                       int elem_bytes, void* stream);

/* A Linear layer's weight and bias gradients in the PPO update under the opt-in bf16 update (the gradients
 * loss.backward() forms for every nn.Linear of actor_critic_dh.py:45-111 at dh_ppo.py:180; replaces the split-K
 * batched GEMM + t1policy_slice_sum + torch's dim-0 bias sum of dh_policy._LinearSplitK.backward):
 *   grad_weight[m, n] (+)= sum_r gy[r, m] x[r, n]   (M x N fp32, row-major)
 *   grad_bias[m]      (+)= sum_r gy[r, m]           (fp32; grad_bias NULL: not formed)
 * accumulate != 0: added to the gradients already there (autograd's accumulation into an existing .grad), else
 * stored.
 * gy (rows, M) and x (rows, N) are row-major bf16 with 4-byte-aligned bases; the sums are fp32 over exact bf16
 * products in a fixed order (deterministic).  workspace: workspace_bytes(rows, M, N) device bytes, 16-byte aligned.
 * Returns 0, -1 on bad arguments, -2 on a launch / device error (workspace_bytes: the size, or -1 / -2). */
long long t1policy_linear_wgrad_workspace_bytes(int rows, int M, int N);
int t1policy_linear_wgrad_bf16(const void* gy, const void* x, int rows, int M, int N, void* workspace,
                               long long workspace_bytes, float* grad_weight, float* grad_bias, int accumulate,
                               void* stream);
/* The same on fp32 gy (rows, M) and x (rows, N) -- the fp32 update, the reference's precision (dh_ppo.py:155-182) --
 * on the matrix cores: each fp32 value split into three bf16 parts, the six part products down to 2^-16 of each
 * product formed by v_mfma_f32_32x32x16_bf16 and summed in fp32 (fp32-class: within 2e-6 of |gy|^T |x| of the fp64 sum
 * in tests/test_gpu_linear_wgrad.py), grad_bias the fp32 sum of gy; the same workspace, accumulate and fixed-order
 * sums (deterministic).  Replaces the fp32 update's split-K batched GEMM + slice sum + bias sum. */
int t1policy_linear_wgrad_f32(const float* gy, const float* x, int rows, int M, int N, void* workspace,
                              long long workspace_bytes, float* grad_weight, float* grad_bias, int accumulate,
                              void* stream);

/* t1policy_linear_wgrad_f32 with x's rows ldx >= N elements apart (a column slice read in place: the state estimator's
 * short history).  Returns 0, -1 on bad arguments (a strided x needs T1_WGRAD_STAGED on), -2 on a launch error. */
int t1policy_linear_wgrad_f32x(const float* gy, const float* x, int ldx, int rows, int M, int N, void* workspace,
                               long long workspace_bytes, float* grad_weight, float* grad_bias, int accumulate,
                               void* stream);

/* The fp32 update's Linear forward and input-gradient GEMMs (t1policy_gemm.hip): C (R, N) = A (R, K) B (N, K)^T
 * (+ bias (N), NULL: none); act 1 then applies ELU (alpha 1), act 2 multiplies by ELU's derivative at the ELU outputs
 * aux (R, N) (1 where aux > 0, else aux + 1; aux NULL otherwise), for row-major fp32 A, B, C -- nn.Linear's forward
 * y = x W^T + b (B = W) and its input gradient gx = gy W (B = W^T) of every layer of actor_critic_dh.py:45-111 in the
 * update (dh_ppo.py:155-182; torch's addmm / mm before).  Each fp32 value split into three bf16 parts, the six part
 * products down to 2^-16 of each product on v_mfma_f32_32x32x16_bf16, fp32 sums in k order (fp32-class; deterministic).
 * Returns 0, -1 on bad arguments, -2 on a launch error. */
int t1policy_gemm_nt_f32(const float* A, const float* B, const float* bias, const float* aux, float* C, int R, int N,
                         int K, int act, void* stream);

/* t1policy_gemm_nt_f32 on strided operands, with no copies for the update's two non-contiguous cases: A rows lda >= K
 * elements apart (a column slice of a wider matrix: the state estimator's short history, obs[:, -235:]), and B either
 * (N, K) rows ldb >= K apart (b_kn = 0) or given as its transpose, (K, N) rows ldb >= N apart (b_kn = 1: the input
 * gradient gx = g W of a Linear reads its weight W (out, in) in place as B = W^T).  The same parts, products and k-order
 * sums as t1policy_gemm_nt_f32.  Each operand's extent below 1 GiB.  Returns 0, -1 on bad arguments, -2 on a launch
 * error. */
int t1policy_gemm_f32(const float* A, int lda, const float* B, int ldb, int b_kn, const float* bias, const float* aux,
                      float* C, int R, int N, int K, int act, void* stream);

/* The PPO minibatch's actor-observation rows from the frame-history rollout storage (not in the reference, whose
 * RolloutStorage keeps every step's whole history: rollout_storage.py:153-173; ti5_isaacgym_amd/algo/rollout.py
 * _HistoryRows restates this in torch):
 *   out[m] = seq[n, k : k + frames] flattened, with the frames of times < first[k, n] zeroed
 *   (k = idx[m] / num_envs, n = idx[m] % num_envs, frame j of the window at time k - frames + 1 + j)
 *   seq   (num_envs, frames + steps - 1, frame), elements of elem_bytes (2: bf16 / fp16, 4: fp32), contiguous
 *   first (steps, num_envs) int64: the first valid time of each step's window; idx (rows) int64 in [0, steps*num_envs)
 *   out   (rows, frames * frame), same element type
 * Returns 0 on success, -1 on bad arguments, -2 on a launch error. */
int t1policy_history_rows(const void* seq, const int64_t* first, const int64_t* idx, void* out, int rows, int num_envs,
                          int steps, int frames, int frame, int elem_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif
