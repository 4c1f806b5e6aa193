// The DH policy's rollout forward after the first history conv, fused into one kernel (include/t1policy.h,
// t1policy_heads_*): every dense layer of actor_critic_dh.py:8-188 the rollout's act() runs --
//
//   long history tail  conv2 (32 -> 16, k4 s2) + ReLU, flatten (16 x 6), 96 -> 128 ELU -> 64      (actor_critic_dh.py:83-96)
//   state estimator    short history (235) -> 256 ELU -> 128 ELU -> 64 ELU -> 3                  (:98-111)
//   actor              [short | estimate | code] (302) -> 512 ELU -> 256 ELU -> 128 ELU -> 12    (:45-58, :163-170)
//   critic             privileged (219) -> 768 ELU -> 256 ELU -> 128 ELU -> 1                   (:60-73, :185-188)
//
// plus the Normal sample, its log-prob and the broadcast sigma (DHPPO._act_body), from the first conv's output
// (t1policy_conv1d_forward_packed), the actor and critic observations and a standard-normal draw.
//
// A workgroup owns 64 envs (k_heads64, the default: two 32-env column tiles sharing every weight fragment, below) or
// 32 (k_heads, A/B) and one role (actor chain or critic), eight waves (two per SIMD) splitting each layer's
// 32-output tiles; every layer is a chain of
// v_mfma_f32_32x32x16_f16 with the WEIGHTS as the A operand (32 output features x 16 inputs) and the ACTIVATIONS as
// the B operand (16 inputs x 32 envs), so a layer's 32 x 32 result has the env on the lane and the features in the
// 16 accumulator registers -- exactly the B fragments of the next layer's two k-steps (permuted k order, cdna guide
// "An accumulator tile as the next MFMA's operand"): an output tile goes to LDS as two 1-KB fragments per precision
// half with one ds_write_b128 each, and the next layer reads them back with one ds_read_b128 each, no transposes.
// The weight fragments are packed once per act() (k_heads_pack) in that permuted k order.
//
// fp32 accuracy from the fp16 matrix cores, as the first conv (t1policy.hip): v = hi + lo / 2^11 with hi = fp16(v),
// lo = fp16((v - hi) 2^11), y = sum hi.hi + 2^-11 sum (hi.lo + lo.hi) in two fp32 accumulators; the dropped lo.lo
// and the residual rounding are ~2^-22 of each product.
//
// Bounds: per 32-env tile the actor chain is 976 step-tiles and the critic 792 (one step-tile = a
// 32 x 16 weight fragment pair = 3 MFMAs, 2 KB of fragments): 3.6 MB of fragments streamed from L2 per tile pair and
// 1.4 M MFMA-cycles per tile pair -- at the XCD L2's ~70 GB/s/CU of shared rows the fragment stream, not the matrix
// cores, sets the time.  Every XCD (blockIdx mod 8) runs both roles, alternating in its dispatch order, so the longer
// actor chain is spread over all CUs; its 4 MB L2 holds both roles' 3.6 MB of fragments.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdlib>

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr float PH_SPLIT = 2048.0f;
constexpr int PH_M = 32;      // envs per workgroup (one MFMA column tile)
// waves per workgroup: 8 = two per SIMD, each with half the output tiles and a shallower fragment ring (act() 0.177 ->
// 0.147 ms at 8192 envs, profiles/r05h8_*); 4 = one per SIMD, the round-4 kernel (A/B)
#ifndef T1_HEADS_WAVES
#define T1_HEADS_WAVES 8
#endif
constexpr int PH_WAVES = T1_HEADS_WAVES;
// 8-wave ring depths (k-steps in flight) for 1, 2 and >= 3 output tiles per wave: act() 0.1419 ms at 4 / 2 / 1 against
// 0.1428 at 6 / 3 / 2, 0.1443 at 8 / 4 / 2 and 0.1470 at 12 / 6 / 2 (profiles/r05hd_act_ab.txt; A/B)
#ifndef T1_HEADS_D1
#define T1_HEADS_D1 4
#endif
#ifndef T1_HEADS_D2
#define T1_HEADS_D2 2
#endif
#ifndef T1_HEADS_D3
#define T1_HEADS_D3 1
#endif
constexpr int PH_OBS_SHORT = 235, PH_CRITIC = 219, PH_Y1 = 14 * 32;
constexpr int PH_NLAYER = 15;
enum { ACT_NONE = 0, ACT_RELU = 1, ACT_ELU = 2 };

// An input segment of a layer's k axis: `steps` k-steps starting at step `s0` map to input columns col0 .. col0 +
// len - 1, in natural order (staged from global memory: element j of lane half h of step s = column 16 (s - s0) +
// 8 h + j) or in the permuted order of an accumulator tile (column 16 (s - s0) + 8 (j >> 2) + 4 h + (j & 3)).
struct Seg {
  int s0, steps, col0, len, perm;
};
struct Layer {
  int n, k, ks, act;  // outputs, inputs (the weight's row length), k-steps, activation
  Seg seg[3];
  int nseg;
};
// layer order = parameter order of t1policy_heads_* (include/t1policy.h)
constexpr Layer PH_L[PH_NLAYER] = {
    // long-history tail: conv2 as a 448 -> 96 Toeplitz layer over the channels-last conv1 output (flatten order
    // o * 6 + l of nn.Flatten on (16, 6)), then the two Linears
    {96, 128, 28, ACT_RELU, {{0, 28, 0, PH_Y1, 0}}, 1},
    {128, 96, 6, ACT_ELU, {{0, 6, 0, 96, 1}}, 1},
    {64, 128, 8, ACT_NONE, {{0, 8, 0, 128, 1}}, 1},
    // state estimator
    {256, PH_OBS_SHORT, 15, ACT_ELU, {{0, 15, 0, PH_OBS_SHORT, 0}}, 1},
    {128, 256, 16, ACT_ELU, {{0, 16, 0, 256, 1}}, 1},
    {64, 128, 8, ACT_ELU, {{0, 8, 0, 128, 1}}, 1},
    {3, 64, 4, ACT_NONE, {{0, 4, 0, 64, 1}}, 1},
    // actor: [short (natural) | estimate (permuted, rows 0..2 of one half-tile) | code (permuted)]
    {512, 302, 20, ACT_ELU, {{0, 15, 0, PH_OBS_SHORT, 0}, {15, 1, 235, 3, 1}, {16, 4, 238, 64, 1}}, 3},
    {256, 512, 32, ACT_ELU, {{0, 32, 0, 512, 1}}, 1},
    {128, 256, 16, ACT_ELU, {{0, 16, 0, 256, 1}}, 1},
    {12, 128, 8, ACT_NONE, {{0, 8, 0, 128, 1}}, 1},
    // critic
    {768, PH_CRITIC, 14, ACT_ELU, {{0, 14, 0, PH_CRITIC, 0}}, 1},
    {256, 768, 48, ACT_ELU, {{0, 48, 0, 768, 1}}, 1},
    {128, 256, 16, ACT_ELU, {{0, 16, 0, 256, 1}}, 1},
    {1, 128, 8, ACT_NONE, {{0, 8, 0, 128, 1}}, 1},
};
constexpr int ph_nt(int l) { return (PH_L[l].n + 31) / 32; }
constexpr int ph_off(int l) {  // first step-tile of layer l in the fragment buffer
  int o = 0;
  for (int i = 0; i < l; ++i) o += ph_nt(i) * PH_L[i].ks;
  return o;
}
constexpr int PH_UNITS = ph_off(PH_NLAYER);          // 1,768 step-tiles
constexpr int ph_toff(int l) {  // first output tile of layer l (bias fragments)
  int o = 0;
  for (int i = 0; i < l; ++i) o += ph_nt(i);
  return o;
}
constexpr int PH_TILES = ph_toff(PH_NLAYER);          // 90 output tiles
// the weight fragments (hi + lo, 64 lanes x 16 B per step-tile), then each output tile's bias in the C/D layout
// (4 x float4 per lane: [tile][quad][lane], register r of lane l = bias of row (r & 3) + 8 (r >> 2) + 4 (l >> 5))
constexpr int PH_WFRAG_BYTES = PH_UNITS * 2 * 64 * 16;  // 3,620,864
constexpr int PH_FRAG_BYTES = PH_WFRAG_BYTES + PH_TILES * 4 * 64 * 16;  // + 368,640

struct PhParams {
  const float* w[PH_NLAYER];
  const float* b[PH_NLAYER];
  const float* std;
};

// the weight element feeding output o from input column col of layer L (conv2 as its Toeplitz matrix)
template <int L>
__device__ __forceinline__ float ph_weight(const PhParams& P, int o, int col) {
  if constexpr (L == 0) {
    const int oc = o / 6, lp = o % 6, p = col >> 5, c = col & 31, t = p - 2 * lp;
    return (t >= 0 && t < 4) ? P.w[0][(oc * 32 + c) * 4 + t] : 0.0f;
  } else {
    return P.w[L][o * PH_L[L].k + col];
  }
}

template <int L>
__device__ __forceinline__ int ph_col(int s, int h, int j) {
  constexpr Layer Y = PH_L[L];
#pragma unroll
  for (int g = 0; g < Y.nseg; ++g) {
    const Seg q = Y.seg[g];
    if (s >= q.s0 && s < q.s0 + q.steps) {
      const int r = 16 * (s - q.s0) + (q.perm ? 8 * (j >> 2) + 4 * h + (j & 3) : 8 * h + j);
      return r < q.len ? q.col0 + r : -1;
    }
  }
  return -1;
}

__device__ __forceinline__ void split8(const float (&v)[8], h8& hi, h8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const _Float16 x = (_Float16)v[j];
    hi[j] = x;
    lo[j] = (_Float16)((v[j] - (float)x) * PH_SPLIT);
  }
}

template <int L>
__device__ __forceinline__ void ph_pack_unit(const PhParams& P, h8* __restrict__ frag, int u, int lane) {
  constexpr Layer Y = PH_L[L];
  const int nt = u / Y.ks, s = u % Y.ks;
  const int o = 32 * nt + (lane & 31), h = lane >> 5;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int col = ph_col<L>(s, h, j);
    v[j] = (o < Y.n && col >= 0) ? ph_weight<L>(P, o, col) : 0.0f;
  }
  h8 hi, lo;
  split8(v, hi, lo);
  const int unit = ph_off(L) + u;
  frag[(unit * 2 + 0) * 64 + lane] = hi;
  frag[(unit * 2 + 1) * 64 + lane] = lo;
}

template <int L>
__device__ __forceinline__ bool ph_pack_dispatch(const PhParams& P, h8* frag, int unit, int lane) {
  if constexpr (L == PH_NLAYER) {
    return false;
  } else {
    if (unit < ph_off(L + 1)) {
      ph_pack_unit<L>(P, frag, unit - ph_off(L), lane);
      return true;
    }
    return ph_pack_dispatch<L + 1>(P, frag, unit, lane);
  }
}

template <int L>
__device__ __forceinline__ bool ph_pack_bias(const PhParams& P, float4* __restrict__ bf, int tile, int lane) {
  if constexpr (L == PH_NLAYER) {
    return false;
  } else {
    if (tile < ph_toff(L + 1)) {
      const int nt = tile - ph_toff(L), h = lane >> 5;
      float v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = 32 * nt + (r & 3) + 8 * (r >> 2) + 4 * h;
        // conv2 (L = 0): one bias per output channel, row = channel * 6 + position (the flatten order)
        v[r] = row < PH_L[L].n ? P.b[L][L == 0 ? row / 6 : row] : 0.0f;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) bf[(tile * 4 + q) * 64 + lane] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
      return true;
    }
    return ph_pack_bias<L + 1>(P, bf, tile, lane);
  }
}

__global__ __launch_bounds__(256) void k_heads_pack(PhParams P, h8* __restrict__ frag) {
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < (PH_UNITS + PH_TILES) * 64; e += gridDim.x * blockDim.x) {
    if (e < PH_UNITS * 64)
      ph_pack_dispatch<0>(P, frag, e >> 6, e & 63);
    else
      ph_pack_bias<0>(P, reinterpret_cast<float4*>(reinterpret_cast<char*>(frag) + PH_WFRAG_BYTES),
                      (e >> 6) - PH_UNITS, e & 63);
  }
}

// ---- the forward kernel
typedef h8 Frag[2][64];  // one k-step of B fragments in LDS: [hi, lo][lane]

struct ActorLds {
  Frag x[20];  // actor input: short history (steps 0..14), estimate (15), history code (16..19)
  Frag p[32];  // 512-wide activations (and the staged conv1 output, 28 steps)
  Frag q[16];  // 256-wide activations
};
struct CriticLds {
  Frag p[48];  // 768-wide activations
  Frag q[16];  // the staged privileged observations (14 steps), then 256-wide activations
};
// split-K on the narrow layers (8 waves): a layer of NT < 8 output tiles deals each tile's k-steps over SK waves
// (NT SK <= 8, at least two k-steps each, SK a power of two); waves kh = 1 .. SK-1 leave their partial 32 x 32 sums
// (hi.hi + 2^-11 (hi.lo + lo.hi), one fp32 per element) in LDS and wave kh = 0 adds them in kh order before the bias
// and the activation.  Measured +-0 (act() 0.1276-0.1292 ms off, 0.1282-0.1298 on, profiles/r07c_act_ab.txt): the
// waves' k chains are not what bounds the kernel, its fragment stream from L2 is, so it stays off (A/B).
#ifndef T1_HEADS_SPLITK
#define T1_HEADS_SPLITK 0
#endif
constexpr int PH_RED_TILES = 4;  // partial tiles in LDS at once: (SK - 1) NT <= 4
constexpr int ph_sk(int l) {
  if (!T1_HEADS_SPLITK || PH_WAVES != 8) return 1;
  const int nt = ph_nt(l), ks = PH_L[l].ks;
  int sk = 1;
  while (nt * sk * 2 <= PH_WAVES && ks % (sk * 2) == 0 && ks / (sk * 2) >= 2 && (sk * 2 - 1) * nt <= PH_RED_TILES)
    sk *= 2;
  return sk;
}
struct PhLds {
  union {
    ActorLds a;
    CriticLds c;
  };
#if T1_HEADS_SPLITK
  float4 red[PH_RED_TILES][4][64];  // split-K partial sums: [(kh - 1) NT + tile][register quad][lane]
#endif
};

#ifndef T1_HEADS_FAST_ELU
#define T1_HEADS_FAST_ELU 1  // act() 0.1336 -> 0.1279 ms at 8192 envs (profiles/r07b_act_ab.txt)
#endif
// expm1(v) for ELU's negative branch, branch-free.  1: the device library's expm1f algorithm (range reduction by
// n = rint(v log2 e) with ln 2 in two parts, the same degree-7 polynomial, 2^n expm1(r) + (2^n - 1)) without its
// overflow and v < -17 fix-ups, which v <= 0 never needs once v is clamped at -88: bit-identical to expm1f there (NaN
// included).
// 2: 2^(v log2 e) - 1 on the hardware exponential below -1/4, a degree-6 Taylor polynomial above (not bit-identical).
__device__ __forceinline__ float ph_expm1_neg(float v) {
#if T1_HEADS_FAST_ELU == 2
  const float e = __builtin_amdgcn_exp2f(v * 1.44269504088896341f) - 1.0f;
  float p = fmaf(v, 1.0f / 720.0f, 1.0f / 120.0f);
  p = fmaf(v, p, 1.0f / 24.0f);
  p = fmaf(v, p, 1.0f / 6.0f);
  p = fmaf(v, p, 0.5f);
  p = fmaf(v * v, p, v);
  return v < -0.25f ? e : p;
#else
  v = v < -88.0f ? -88.0f : v;  // (not fmaxf: a NaN stays a NaN, as in expm1f and torch's ELU)
  const float n = __builtin_rintf(v * __builtin_bit_cast(float, 0x3fb8aa3bu));
  float r = fmaf(n, __builtin_bit_cast(float, 0xbf317218u), v);
  r = fmaf(n, __builtin_bit_cast(float, 0x3102e308u), r);
  float p = fmaf(r, __builtin_bit_cast(float, 0x395133b1u), __builtin_bit_cast(float, 0x3ab69700u));
  p = fmaf(r, p, __builtin_bit_cast(float, 0x3c0887f9u));
  p = fmaf(r, p, __builtin_bit_cast(float, 0x3d2aaa81u));
  p = fmaf(r, p, __builtin_bit_cast(float, 0x3e2aaaabu));
  p = fmaf(r, p, 0.5f);
  p = r * p;
  const float m = fmaf(r, p, r);  // expm1(r)
  const float t = __builtin_ldexpf(1.0f, (int)n);
  return fmaf(t, m, t - 1.0f);
#endif
}

__device__ __forceinline__ float ph_act(float v, int act) {
  if (act == ACT_RELU) return v > 0.0f ? v : 0.0f;
#ifdef T1_HEADS_WHATIF_NOELU  // timing-only what-if build: ELU as ReLU
  if (act == ACT_ELU) return v > 0.0f ? v : 0.0f;
#else
#if T1_HEADS_FAST_ELU && defined(T1_HEADS_ELU_BRANCH)  // A/B: the expm1 under a branch per value (hipcc's choice)
  if (act == ACT_ELU) return v > 0.0f ? v : ph_expm1_neg(v);
#elif T1_HEADS_FAST_ELU
  if (act == ACT_ELU) {  // branch-free: expm1 of min(v, 0) (a NaN passes through), then the select
    const float e = ph_expm1_neg(v > 0.0f ? 0.0f : v);
    return v > 0.0f ? v : e;
  }
#else
  if (act == ACT_ELU) return v > 0.0f ? v : expm1f(v);
#endif
#endif
  return v;
}

// stage `steps` k-steps of natural-order B fragments from rows of global memory: element j of lane (r, h) of step s
// = src[env r][col0 + 16 s + 8 h + j] (0 past len or past the batch), split into hi / lo.  Steps round-robin over the
// waves.
template <bool RELU>
__device__ __forceinline__ void ph_stage(Frag* dst, int steps, const float* __restrict__ src, long long stride,
                                         int col0, int len, int env, bool live, int wave, int lane) {
  const int h = lane >> 5;
  const float* row = src + (long long)env * stride + col0;
  for (int s = wave; s < steps; s += PH_WAVES) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = 16 * s + 8 * h + j;
      // (non-temporal loads here, so the once-read inputs would not evict fragments: act() 0.129 -> 0.153 ms, r07c)
      float x = (live && c < len) ? row[c] : 0.0f;
      v[j] = RELU ? (x > 0.0f ? x : 0.0f) : x;
    }
    h8 hi, lo;
    split8(v, hi, lo);
    dst[s][0][lane] = hi;
    dst[s][1][lane] = lo;
  }
}

enum { OUT_LDS = 0, OUT_LDS_HALF = 1, OUT_MEAN = 2, OUT_VALUE = 3 };

struct PhOut {  // the global outputs (OUT_MEAN / OUT_VALUE layers)
  const float* eps;
  const float* std;
  float* mean;
  float* actions;
  float* sigma;
  float* logp;
  float* value;
  int env;
  bool live;
};

// one dense layer for this wave's output tiles nt = wave + PH_WAVES i: B fragments from `in` (LDS), A fragments streamed
// from the packed buffer, result + bias through the activation into `out` (LDS, k-steps out0 + 2 nt + {0, 1}) or the
// global outputs.  Waves past the layer's tile count skip the products and store nothing.
// the weight-fragment register ring of layer L: its loads run D k-steps ahead of their MFMAs through D + 1 slots
// (about 16 x 96 MFMA cycles of cover over an L2 hit under load); its first D steps are issued during the previous
// layer (ph_prologue), so no layer starts on an empty pipeline
template <int L> struct PhRing {
  static constexpr int NT = ph_nt(L), KS = PH_L[L].ks, SK = ph_sk(L), KL = KS / SK;
  static constexpr int T = SK > 1 ? 1 : (NT + PH_WAVES - 1) / PH_WAVES;
  // the wave's output tile i and the first of its KL k-steps (idle waves: a valid tile, loaded and never used)
  static __device__ __forceinline__ int tile(int wave, int i) {
    if constexpr (SK > 1) return wave % NT;
    return (wave + PH_WAVES * i) < NT ? wave + PH_WAVES * i : NT - 1;
  }
  static __device__ __forceinline__ int kpart(int wave) { return SK > 1 && wave < NT * SK ? wave / NT : 0; }
  static __device__ __forceinline__ bool busy(int wave) { return PH_WAVES == 4 || wave < NT * SK; }
  // two waves per SIMD (PH_WAVES 8): the other wave covers part of the latency, and 256 VGPRs hold the accumulators
  // and a ring of 1-4 steps (4 waves: 512 registers, 4-16 steps)
  static constexpr int D0 = PH_WAVES == 8 ? (T >= 3 ? T1_HEADS_D3 : (T >= 2 ? T1_HEADS_D2 : T1_HEADS_D1))
                                          : (T >= 4 ? 4 : (T >= 2 ? 8 : 16));
  static constexpr int D = D0 < KL ? D0 : KL - 1;
  static constexpr int R = D + 1;
  h8 w[R][T][2];
};
template <int L>
__device__ __forceinline__ void ph_load(const h8* __restrict__ frag, PhRing<L>& rg, int slot, int s, int wave,
                                        int lane) {
  typedef PhRing<L> G;
  constexpr int OFF = ph_off(L);
  const int ks = G::kpart(wave) * G::KL + s;  // s counts the wave's own k-steps
#pragma unroll
  for (int i = 0; i < G::T; ++i) {
    const int nt = G::tile(wave, i);
#ifdef T1_HEADS_WHATIF_NOLOAD  // timing-only what-if build: every fragment load hits the same 2 KB (L1)
    const h8* w = frag + lane + (size_t)(((OFF + nt * G::KS + ks) & 0) * 2) * 64;
#else
    const h8* w = frag + lane + (size_t)((OFF + nt * G::KS + ks) * 2) * 64;
#endif
    rg.w[slot][i][0] = w[0];
    rg.w[slot][i][1] = w[64];
  }
}
template <int L>
__device__ __forceinline__ void ph_prologue(const h8* __restrict__ frag, PhRing<L>& rg, int wave, int lane) {
#pragma clang loop unroll(full)
  for (int s = 0; s < PhRing<L>::D; ++s) ph_load<L>(frag, rg, s, s, wave, lane);
}

// one dense layer for this wave's output tiles nt = wave + PH_WAVES i: B fragments from `in` (LDS), A fragments through
// the ring rg (prologue already issued), result + bias through the activation into `out` (LDS, k-steps
// out0 + 2 nt + {0, 1}) or the global outputs.  LN >= 0: layer LN's prologue is issued into *nx before this layer's
// epilogue.  Waves past the layer's tile count (8 waves, layers of < 8 tiles) skip the products and store nothing;
// at 4 waves every layer has a tile per wave except the narrow heads, whose spare waves recompute the last tile.
template <int L, int OUT, int LN>
__device__ __forceinline__ void ph_layer(const h8* __restrict__ frag, const PhParams& P, const Frag* in, Frag* out,
                                         int out0, const PhOut& G, int wave, int lane, PhRing<L>& rg,
                                         PhRing<(LN < 0 ? L : LN)>* nx, float4 (*red)[4][64]) {
  constexpr Layer Y = PH_L[L];
  typedef PhRing<L> RG;
  constexpr int NT = RG::NT, KL = RG::KL, SK = RG::SK, T = RG::T, D = RG::D, R = RG::R;
  const int h = lane >> 5;
  const int k0 = RG::kpart(wave) * KL;  // the wave's first k-step (split-K), wave-uniform
  f16v acc0[T], acc1[T];
#pragma unroll
  for (int i = 0; i < T; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc0[i][r] = acc1[i][r] = 0.0f;
  float4 bias[T][4];
  h8 bq[2][2];
  bq[0][0] = in[k0][0][lane];
  bq[0][1] = in[k0][1][lane];
  // a wave past the layer's tiles x k parts (PH_WAVES 8 on the narrow layers) skips the K loop (it stores nothing)
  if (RG::busy(wave))
#pragma clang loop unroll(full)
  for (int s = 0; s < KL; ++s) {
    if (s + D < KL) ph_load<L>(frag, rg, (s + D) % R, s + D, wave, lane);
    if (s == KL - 1 - D) {  // the bias fragments behind the layer's last weight loads (no drain at the epilogue)
      const float4* bf = reinterpret_cast<const float4*>(reinterpret_cast<const char*>(frag) + PH_WFRAG_BYTES);
#pragma unroll
      for (int i = 0; i < T; ++i) {
        const int nt = RG::tile(wave, i);
#pragma unroll
        for (int q = 0; q < 4; ++q) bias[i][q] = bf[((ph_toff(L) + nt) * 4 + q) * 64 + lane];
      }
    }
    if (s + 1 < KL) {
      bq[(s + 1) & 1][0] = in[k0 + s + 1][0][lane];
      bq[(s + 1) & 1][1] = in[k0 + s + 1][1][lane];
    }
    __builtin_amdgcn_sched_barrier(0);
    const h8 bh = bq[s & 1][0], bl = bq[s & 1][1];
#pragma unroll
    for (int i = 0; i < T; ++i) {
      const h8 ah = rg.w[s % R][i][0], al = rg.w[s % R][i][1];
#ifdef T1_HEADS_WHATIF_NOMFMA  // timing-only what-if build: one MFMA per step-tile instead of three
      acc0[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah + al, bh + bl, acc0[i], 0, 0, 0);
#else
      acc0[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc0[i], 0, 0, 0);
      acc1[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc1[i], 0, 0, 0);
      acc1[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc1[i], 0, 0, 0);
#endif
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (LN >= 0) ph_prologue<LN>(frag, *nx, wave, lane);  // the next layer's first fragments in flight
  float y[T][16];  // hi.hi + 2^-11 (hi.lo + lo.hi) per element, then the split-K partials in k order
#pragma unroll
  for (int i = 0; i < T; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) y[i][r] = acc0[i][r] + acc1[i][r] * (1.0f / PH_SPLIT);
  if constexpr (SK > 1) {
    const int kh = RG::kpart(wave);
    if (RG::busy(wave) && kh > 0) {
      float4(*dst)[64] = red[(kh - 1) * NT + wave % NT];
#pragma unroll
      for (int q = 0; q < 4; ++q) dst[q][lane] = make_float4(y[0][4 * q], y[0][4 * q + 1], y[0][4 * q + 2], y[0][4 * q + 3]);
    }
    __syncthreads();  // every wave: the partials in LDS
    if (wave < NT) {
#pragma unroll
      for (int p = 1; p < SK; ++p) {
        const float4(*src)[64] = red[(p - 1) * NT + wave];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 u = src[q][lane];
          y[0][4 * q] += u.x; y[0][4 * q + 1] += u.y; y[0][4 * q + 2] += u.z; y[0][4 * q + 3] += u.w;
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < T; ++i) {
    const int nt = wave + PH_WAVES * i;
    if (nt >= NT) break;  // wave-uniform (split-K: the kh = 0 waves, 0 .. NT - 1)
    float v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float4 b4 = bias[i][r >> 2];
      const float b = (r & 3) == 0 ? b4.x : (r & 3) == 1 ? b4.y : (r & 3) == 2 ? b4.z : b4.w;
      v[r] = ph_act(y[i][r] + b, Y.act);
    }
    if constexpr (OUT == OUT_LDS || OUT == OUT_LDS_HALF) {
#pragma unroll
      for (int s = 0; s < (OUT == OUT_LDS ? 2 : 1); ++s) {
        float u[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) u[j] = v[8 * s + j];
        h8 hi, lo;
        split8(u, hi, lo);
        out[out0 + 2 * nt + s][0][lane] = hi;
        out[out0 + 2 * nt + s][1][lane] = lo;
      }
    } else if constexpr (OUT == OUT_MEAN) {
      // the Normal sample a = mean + sigma eps and its log-prob, summed over the 12 actions (DHPPO._act_body;
      // torch.distributions.Normal.log_prob): rows 0-3, 8-11 on lane half 0, rows 4-7 on half 1
      float lp = 0.0f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row < Y.n && G.live) {
          const float sd = G.std[row];
          const size_t ix = (size_t)G.env * Y.n + row;
          const float a = v[r] + sd * G.eps[ix];
          const float d = a - v[r];
          lp += -(d * d) / (2.0f * (sd * sd)) - logf(sd) - 0.91893853320467274178f;  // log(sqrt(2 pi))
          G.mean[ix] = v[r];
          G.actions[ix] = a;
          G.sigma[ix] = sd;
        }
      }
      lp += __shfl_xor(lp, 32);
      if (h == 0 && G.live) G.logp[G.env] = lp;
    } else {
      if (h == 0 && G.live) G.value[G.env] = v[0];
    }
  }
}

__global__ __launch_bounds__(64 * PH_WAVES) __attribute__((amdgpu_waves_per_eu(PH_WAVES / 4, PH_WAVES / 4)))
void k_heads(PhParams P, const h8* __restrict__ frag, const float* __restrict__ y1, const float* __restrict__ obs,
             int obs_cols, const float* __restrict__ cobs, int cobs_cols, PhOut G, int batch, int xcd_split) {
  __shared__ PhLds S;
#if T1_HEADS_SPLITK
  float4(*red)[4][64] = S.red;
#else
  float4(*red)[4][64] = nullptr;
#endif
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  // role and tile: blockIdx mod 8 is the XCD; actor tiles on XCDs 0-3, critic tiles on 4-7 (xcd_split), else
  // alternating
  const int bid = blockIdx.x;
  // xcd_split 2: both roles on every XCD, alternating in each XCD's dispatch order (a CU's two workgroups tend to be
  // one actor chain and one critic; each L2 then holds both roles' 3.6 MB of fragments)
  const bool critic = xcd_split == 2 ? ((bid >> 3) & 1) != 0 : (xcd_split ? (bid & 4) != 0 : (bid & 1) != 0);
  const int tile = xcd_split == 2 ? ((bid >> 4) << 3) + (bid & 7) : (xcd_split ? (bid >> 3) * 4 + (bid & 3) : bid >> 1);
  const int env0 = tile * PH_M;
  if (env0 >= batch) return;
  const int env = env0 + (lane & 31);
  const bool live = env < batch;
  const int envc = live ? env : batch - 1;
  G.env = envc;
  G.live = live;
  if (!critic) {
    ActorLds& A = S.a;
    ph_stage<true>(A.p, 28, y1, PH_Y1, 0, PH_Y1, envc, live, wave, lane);                       // relu(conv1)
    ph_stage<false>(A.x, 15, obs, obs_cols, obs_cols - PH_OBS_SHORT, PH_OBS_SHORT, envc, live, wave, lane);
    PhRing<0> g0;
    ph_prologue<0>(frag, g0, wave, lane);  // the first layer's fragments load across the barrier
    __syncthreads();
    PhRing<1> g1;
    ph_layer<0, OUT_LDS, 1>(frag, P, A.p, A.q, 0, G, wave, lane, g0, &g1, red);
    __syncthreads();
    PhRing<2> g2;
    ph_layer<1, OUT_LDS, 2>(frag, P, A.q, A.p, 0, G, wave, lane, g1, &g2, red);
    __syncthreads();
    PhRing<3> g3;
    ph_layer<2, OUT_LDS, 3>(frag, P, A.p, A.x, 16, G, wave, lane, g2, &g3, red);  // history code -> actor input 16..19
    PhRing<4> g4;
    ph_layer<3, OUT_LDS, 4>(frag, P, A.x, A.q, 0, G, wave, lane, g3, &g4, red);  // reads steps 0..14 only: no barrier
    __syncthreads();
    PhRing<5> g5;
    ph_layer<4, OUT_LDS, 5>(frag, P, A.q, A.p, 0, G, wave, lane, g4, &g5, red);
    __syncthreads();
    PhRing<6> g6;
    ph_layer<5, OUT_LDS, 6>(frag, P, A.p, A.q, 0, G, wave, lane, g5, &g6, red);
    __syncthreads();
    PhRing<7> g7;
    ph_layer<6, OUT_LDS_HALF, 7>(frag, P, A.q, A.x, 15, G, wave, lane, g6, &g7, red);  // estimate -> actor input 15
    __syncthreads();
    PhRing<8> g8;
    ph_layer<7, OUT_LDS, 8>(frag, P, A.x, A.p, 0, G, wave, lane, g7, &g8, red);
    __syncthreads();
    PhRing<9> g9;
    ph_layer<8, OUT_LDS, 9>(frag, P, A.p, A.q, 0, G, wave, lane, g8, &g9, red);
    __syncthreads();
    PhRing<10> g10;
    ph_layer<9, OUT_LDS, 10>(frag, P, A.q, A.p, 0, G, wave, lane, g9, &g10, red);
    __syncthreads();
    ph_layer<10, OUT_MEAN, -1>(frag, P, A.p, nullptr, 0, G, wave, lane, g10, nullptr, red);
  } else {
    CriticLds& C = S.c;
    ph_stage<false>(C.q, 14, cobs, cobs_cols, 0, PH_CRITIC, envc, live, wave, lane);
    PhRing<11> g11;
    ph_prologue<11>(frag, g11, wave, lane);
    __syncthreads();
    PhRing<12> g12;
    ph_layer<11, OUT_LDS, 12>(frag, P, C.q, C.p, 0, G, wave, lane, g11, &g12, red);
    __syncthreads();
    PhRing<13> g13;
    ph_layer<12, OUT_LDS, 13>(frag, P, C.p, C.q, 0, G, wave, lane, g12, &g13, red);
    __syncthreads();
    PhRing<14> g14;
    ph_layer<13, OUT_LDS, 14>(frag, P, C.q, C.p, 0, G, wave, lane, g13, &g14, red);
    __syncthreads();
    ph_layer<14, OUT_VALUE, -1>(frag, P, C.p, nullptr, 0, G, wave, lane, g14, nullptr, red);
  }
}

// ---- 64 envs per workgroup (k_heads64, the default; T1POLICY_HEADS64=0: the 32-env k_heads above, A/B).  At 32 envs
// a workgroup takes ~42 us whether 256 or 512 of them run (4096 / 8192 envs, profiles/r07e), and its 139 KB of LDS
// leaves one per CU, so 8192 envs take two rounds.  Here each weight fragment feeds BOTH 32-env column tiles (six
// MFMAs per step-tile instead of three, the same fragment stream per workgroup), so 8192 envs take one round.  The LDS
// holds 64 envs' activations in 144 KB because no layer output wider than 256 is ever resident: the actor's 512-wide
// layer runs in two halves of 8 output tiles and the critic's 768-wide one in three, each half / third feeding the
// next layer's accumulators (held in registers across the calls) before the next one overwrites it; the short
// history is staged twice (the estimator's first layer, then the actor's).  Every layer call has one output tile per
// wave (8 waves, T = 1).
typedef h8 Frag2[2][2][64];  // one k-step of B fragments of both 32-env tiles: [env tile][hi, lo][lane]
struct Heads64Lds {
  Frag2 px[36];  // actor: PX[0..35]; critic: PX[0..31] (layout per phase in k_heads64)
};

// one layer call: layer L's output tiles [TB, TB + 8) (or to the layer's last tile) over its k-steps [KB, KE)
template <int L_, int KB_, int KE_, int TB_> struct P6Ring {
  static constexpr int L = L_, KB = KB_, KE = KE_, TB = TB_;
  static constexpr int NTL = ph_nt(L), TE = TB + PH_WAVES < NTL ? TB + PH_WAVES : NTL, NW = TE - TB;
  static constexpr int KL = KE - KB, D = T1_HEADS_D1 < KL ? T1_HEADS_D1 : KL - 1, R = D + 1;
  static_assert(PH_WAVES == 8 && KL >= 1 && NW >= 1 && KE <= PH_L[L].ks, "one output tile per wave");
  static __device__ __forceinline__ int tile(int wave) { return wave < NW ? TB + wave : TE - 1; }
  h8 w[R][2];
};
struct P6None {
  static constexpr int L = -1;
};
template <class RG>
__device__ __forceinline__ void ph6_load(const h8* __restrict__ frag, RG& rg, int slot, int s, int wave, int lane) {
  const h8* w = frag + lane + (size_t)((ph_off(RG::L) + RG::tile(wave) * PH_L[RG::L].ks + RG::KB + s) * 2) * 64;
  rg.w[slot][0] = w[0];
  rg.w[slot][1] = w[64];
}
template <class RG>
__device__ __forceinline__ void ph6_prologue(const h8* __restrict__ frag, RG& rg, int wave, int lane) {
#pragma clang loop unroll(full)
  for (int s = 0; s < RG::D; ++s) ph6_load(frag, rg, s, s, wave, lane);
}

struct PhOut64 {  // the global outputs and the workgroup's envs
  const float* eps;
  const float* std;
  float* mean;
  float* actions;
  float* sigma;
  float* logp;
  float* value;
  int env0;
  int batch;
};

// staging as ph_stage, for both env tiles: element j of lane (r, h) of step s, tile et = src[env0 + 32 et + r][col0 +
// 16 s + 8 h + j]
template <bool RELU>
__device__ __forceinline__ void ph6_stage(Frag2* dst, int steps, const float* __restrict__ src, long long stride,
                                          int col0, int len, int env0, int batch, int wave, int lane) {
  const int h = lane >> 5;
  for (int s = wave; s < steps; s += PH_WAVES) {
#pragma unroll
    for (int et = 0; et < 2; ++et) {
      const int env = env0 + 32 * et + (lane & 31);
      const bool live = env < batch;
      const float* row = src + (long long)(live ? env : batch - 1) * stride + col0;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = 16 * s + 8 * h + j;
        const float x = (live && c < len) ? row[c] : 0.0f;
        v[j] = RELU ? (x > 0.0f ? x : 0.0f) : x;
      }
      h8 hi, lo;
      split8(v, hi, lo);
      dst[s][et][0][lane] = hi;
      dst[s][et][1][lane] = lo;
    }
  }
}

// one layer call (see P6Ring): B fragments in[0 .. KL) from LDS, A fragments through the ring rg (prologue issued by the
// previous call), six MFMAs per k-step into acc (ZERO: start from 0; the caller owns acc, so a layer split over calls
// keeps its sums); EPI: result + bias through the activation into out (k-steps out0 + 2 (tile - TB) + {0, 1}) or the
// global outputs.  NX: the next call's ring, whose first fragments are issued before this call's epilogue.
template <class RG, int OUT, bool ZERO, bool EPI, class NX>
__device__ __forceinline__ void ph6_call(const h8* __restrict__ frag, const Frag2* in, Frag2* out, int out0,
                                         const PhOut64& G, int wave, int lane, RG& rg, NX* nx, f16v (&acc0)[2],
                                         f16v (&acc1)[2]) {
  constexpr Layer Y = PH_L[RG::L];
  constexpr int KL = RG::KL, D = RG::D, R = RG::R;
  const int h = lane >> 5;
  const bool busy = wave < RG::NW;  // wave-uniform
  if constexpr (ZERO) {
#pragma unroll
    for (int et = 0; et < 2; ++et)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc0[et][r] = acc1[et][r] = 0.0f;
  }
  float4 bias[4];
  h8 bq[2][2][2];  // [buffer][env tile][hi, lo]
#pragma unroll
  for (int et = 0; et < 2; ++et) {
    bq[0][et][0] = in[0][et][0][lane];
    bq[0][et][1] = in[0][et][1][lane];
  }
  if (busy)
#pragma clang loop unroll(full)
    for (int s = 0; s < KL; ++s) {
      if (s + D < KL) ph6_load(frag, rg, (s + D) % R, s + D, wave, lane);
      if (EPI && s == KL - 1 - D) {  // the bias fragments behind the call's last weight loads
        const float4* bf = reinterpret_cast<const float4*>(reinterpret_cast<const char*>(frag) + PH_WFRAG_BYTES);
#pragma unroll
        for (int q = 0; q < 4; ++q) bias[q] = bf[((ph_toff(RG::L) + RG::tile(wave)) * 4 + q) * 64 + lane];
      }
      if (s + 1 < KL) {
#pragma unroll
        for (int et = 0; et < 2; ++et) {
          bq[(s + 1) & 1][et][0] = in[s + 1][et][0][lane];
          bq[(s + 1) & 1][et][1] = in[s + 1][et][1][lane];
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      const h8 ah = rg.w[s % R][0], al = rg.w[s % R][1];
#pragma unroll
      for (int et = 0; et < 2; ++et) {
        const h8 bh = bq[s & 1][et][0], bl = bq[s & 1][et][1];
        acc0[et] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc0[et], 0, 0, 0);
        acc1[et] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc1[et], 0, 0, 0);
        acc1[et] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc1[et], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  if constexpr (NX::L >= 0) ph6_prologue(frag, *nx, wave, lane);  // the next call's first fragments in flight
  if constexpr (EPI) {
    if (!busy) return;
    const int nt = RG::TB + wave;
#pragma unroll
    for (int et = 0; et < 2; ++et) {
      float v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float4 b4 = bias[r >> 2];
        const float b = (r & 3) == 0 ? b4.x : (r & 3) == 1 ? b4.y : (r & 3) == 2 ? b4.z : b4.w;
        v[r] = ph_act(acc0[et][r] + acc1[et][r] * (1.0f / PH_SPLIT) + b, Y.act);
      }
      const int env = G.env0 + 32 * et + (lane & 31);
      const bool live = env < G.batch;
      if constexpr (OUT == OUT_LDS || OUT == OUT_LDS_HALF) {
#pragma unroll
        for (int s = 0; s < (OUT == OUT_LDS ? 2 : 1); ++s) {
          float u[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) u[j] = v[8 * s + j];
          h8 hi, lo;
          split8(u, hi, lo);
          out[out0 + 2 * (nt - RG::TB) + s][et][0][lane] = hi;
          out[out0 + 2 * (nt - RG::TB) + s][et][1][lane] = lo;
        }
      } else if constexpr (OUT == OUT_MEAN) {  // as ph_layer's OUT_MEAN
        float lp = 0.0f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
          if (row < Y.n && live) {
            const float sd = G.std[row];
            const size_t ix = (size_t)env * Y.n + row;
            const float a = v[r] + sd * G.eps[ix];
            const float d = a - v[r];
            lp += -(d * d) / (2.0f * (sd * sd)) - logf(sd) - 0.91893853320467274178f;  // log(sqrt(2 pi))
            G.mean[ix] = v[r];
            G.actions[ix] = a;
            G.sigma[ix] = sd;
          }
        }
        lp += __shfl_xor(lp, 32);
        if (h == 0 && live) G.logp[env] = lp;
      } else {
        if (h == 0 && live) G.value[env] = v[0];
      }
    }
  }
}

template <int L, int KB, int KE, int TB = 0> using R6 = P6Ring<L, KB, KE, TB>;
template <int L> using R6F = P6Ring<L, 0, PH_L[L].ks, 0>;  // a whole layer

__global__ __launch_bounds__(64 * PH_WAVES) __attribute__((amdgpu_waves_per_eu(PH_WAVES / 4, PH_WAVES / 4)))
void k_heads64(const h8* __restrict__ frag, const float* __restrict__ y1, const float* __restrict__ obs, int obs_cols,
               const float* __restrict__ cobs, int cobs_cols, PhOut64 G, int batch) {
  __shared__ Heads64Lds S;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  // both roles on every XCD (blockIdx mod 8), alternating in each XCD's dispatch order (k_heads' xcd_split 2)
  const int bid = blockIdx.x;
  const bool critic = ((bid >> 3) & 1) != 0;
  const int tile = ((bid >> 4) << 3) + (bid & 7);
  G.env0 = tile * 64;
  G.batch = batch;
  if (G.env0 >= batch) return;
  Frag2* X = S.px;
  f16v a0[2], a1[2];  // the current call's accumulators
  f16v b0[2], b1[2];  // the layer after a split one: its sums across the split layer's calls
  if (!critic) {
    // PX[0..27] the relu'd conv1 output; L0 -> PX[28..33]; L1 -> PX[0..7]; short history -> PX[16..30]; L2 (the
    // history code) -> PX[32..35]; L3 -> PX[0..15]; L4 -> PX[16..23]; L5 -> PX[0..3]; L6 (the estimate) -> PX[31];
    // short history again -> PX[16..30]; the actor input is PX[16..35]; L7 halves -> PX[0..15], each into L8's sums;
    // L8 -> PX[16..31]; L9 -> PX[0..7]; L10 -> the outputs
    ph6_stage<true>(X, 28, y1, PH_Y1, 0, PH_Y1, G.env0, batch, wave, lane);
    R6F<0> g0;
    ph6_prologue(frag, g0, wave, lane);
    __syncthreads();
    R6F<1> g1;
    ph6_call<R6F<0>, OUT_LDS, true, true>(frag, X, X, 28, G, wave, lane, g0, &g1, a0, a1);
    __syncthreads();
    R6F<2> g2;
    ph6_call<R6F<1>, OUT_LDS, true, true>(frag, X + 28, X, 0, G, wave, lane, g1, &g2, a0, a1);
    __syncthreads();
    ph6_stage<false>(X + 16, 15, obs, obs_cols, obs_cols - PH_OBS_SHORT, PH_OBS_SHORT, G.env0, batch, wave, lane);
    R6F<3> g3;
    ph6_call<R6F<2>, OUT_LDS, true, true>(frag, X, X, 32, G, wave, lane, g2, &g3, a0, a1);
    __syncthreads();
    R6F<4> g4;
    ph6_call<R6F<3>, OUT_LDS, true, true>(frag, X + 16, X, 0, G, wave, lane, g3, &g4, a0, a1);
    __syncthreads();
    R6F<5> g5;
    ph6_call<R6F<4>, OUT_LDS, true, true>(frag, X, X, 16, G, wave, lane, g4, &g5, a0, a1);
    __syncthreads();
    R6F<6> g6;
    ph6_call<R6F<5>, OUT_LDS, true, true>(frag, X + 16, X, 0, G, wave, lane, g5, &g6, a0, a1);
    __syncthreads();
    R6<7, 0, 20, 0> g7a;
    ph6_call<R6F<6>, OUT_LDS_HALF, true, true>(frag, X, X, 31, G, wave, lane, g6, &g7a, a0, a1);
    ph6_stage<false>(X + 16, 15, obs, obs_cols, obs_cols - PH_OBS_SHORT, PH_OBS_SHORT, G.env0, batch, wave, lane);
    __syncthreads();
    R6<8, 0, 16> g8a;
    ph6_call<R6<7, 0, 20, 0>, OUT_LDS, true, true>(frag, X + 16, X, 0, G, wave, lane, g7a, &g8a, a0, a1);
    __syncthreads();
    R6<7, 0, 20, 8> g7b;
    ph6_call<R6<8, 0, 16>, OUT_LDS, true, false>(frag, X, nullptr, 0, G, wave, lane, g8a, &g7b, b0, b1);
    __syncthreads();
    R6<8, 16, 32> g8b;
    ph6_call<R6<7, 0, 20, 8>, OUT_LDS, true, true>(frag, X + 16, X, 0, G, wave, lane, g7b, &g8b, a0, a1);
    __syncthreads();
    R6F<9> g9;
    ph6_call<R6<8, 16, 32>, OUT_LDS, false, true>(frag, X, X, 16, G, wave, lane, g8b, &g9, b0, b1);
    __syncthreads();
    R6F<10> g10;
    ph6_call<R6F<9>, OUT_LDS, true, true>(frag, X + 16, X, 0, G, wave, lane, g9, &g10, a0, a1);
    __syncthreads();
    ph6_call<R6F<10>, OUT_MEAN, true, true, P6None>(frag, X, nullptr, 0, G, wave, lane, g10, nullptr, a0, a1);
  } else {
    // PX[16..29] the privileged observations; L11 thirds -> PX[0..15], each into L12's sums; L12 -> PX[16..31];
    // L13 -> PX[0..7]; L14 -> the value
    ph6_stage<false>(X + 16, 14, cobs, cobs_cols, 0, PH_CRITIC, G.env0, batch, wave, lane);
    R6<11, 0, 14, 0> g11a;
    ph6_prologue(frag, g11a, wave, lane);
    __syncthreads();
    R6<12, 0, 16> g12a;
    ph6_call<R6<11, 0, 14, 0>, OUT_LDS, true, true>(frag, X + 16, X, 0, G, wave, lane, g11a, &g12a, a0, a1);
    __syncthreads();
    R6<11, 0, 14, 8> g11b;
    ph6_call<R6<12, 0, 16>, OUT_LDS, true, false>(frag, X, nullptr, 0, G, wave, lane, g12a, &g11b, b0, b1);
    __syncthreads();
    R6<12, 16, 32> g12b;
    ph6_call<R6<11, 0, 14, 8>, OUT_LDS, true, true>(frag, X + 16, X, 0, G, wave, lane, g11b, &g12b, a0, a1);
    __syncthreads();
    R6<11, 0, 14, 16> g11c;
    ph6_call<R6<12, 16, 32>, OUT_LDS, false, false>(frag, X, nullptr, 0, G, wave, lane, g12b, &g11c, b0, b1);
    __syncthreads();
    R6<12, 32, 48> g12c;
    ph6_call<R6<11, 0, 14, 16>, OUT_LDS, true, true>(frag, X + 16, X, 0, G, wave, lane, g11c, &g12c, a0, a1);
    __syncthreads();
    R6F<13> g13;
    ph6_call<R6<12, 32, 48>, OUT_LDS, false, true>(frag, X, X, 16, G, wave, lane, g12c, &g13, b0, b1);
    __syncthreads();
    R6F<14> g14;
    ph6_call<R6F<13>, OUT_LDS, true, true>(frag, X + 16, X, 0, G, wave, lane, g13, &g14, a0, a1);
    __syncthreads();
    ph6_call<R6F<14>, OUT_VALUE, true, true, P6None>(frag, X, nullptr, 0, G, wave, lane, g14, nullptr, a0, a1);
  }
}

bool ph_params(const uint64_t* params, PhParams& P) {
  for (int l = 0; l < PH_NLAYER; ++l) {
    P.w[l] = reinterpret_cast<const float*>(params[2 * l]);
    P.b[l] = reinterpret_cast<const float*>(params[2 * l + 1]);
    if (!P.w[l] || !P.b[l]) return false;
  }
  P.std = reinterpret_cast<const float*>(params[2 * PH_NLAYER]);
  return P.std != nullptr;
}

// the parameter shapes the kernels are compiled for: (out, in) per layer, conv2 as (16, 32 * 4)
bool ph_dims_match(const int* dims) {
  static const int want[PH_NLAYER][2] = {{16, 128}, {128, 96}, {64, 128}, {256, 235}, {128, 256}, {64, 128}, {3, 64},
                                         {512, 302}, {256, 512}, {128, 256}, {12, 128}, {768, 219}, {256, 768},
                                         {128, 256}, {1, 128}};
  for (int l = 0; l < PH_NLAYER; ++l)
    if (dims[2 * l] != want[l][0] || dims[2 * l + 1] != want[l][1]) return false;
  return true;
}

}  // namespace

extern "C" {

int t1policy_heads_frag_bytes(void) { return PH_FRAG_BYTES; }

int t1policy_heads_pack(const uint64_t* params, const int* dims, void* frag, void* stream) {
  if (!params || !dims || !frag) return -1;
  if (!ph_dims_match(dims)) return 1;
  if ((reinterpret_cast<uintptr_t>(frag) & 15u) != 0) return -1;
  PhParams P;
  if (!ph_params(params, P)) return -1;
  hipLaunchKernelGGL(k_heads_pack, dim3(((PH_UNITS + PH_TILES) * 64 + 255) / 256), dim3(256), 0, (hipStream_t)stream, P,
                     reinterpret_cast<h8*>(frag));
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int t1policy_heads_forward(const uint64_t* params, const int* dims, const void* frag, const float* y1,
                           const float* obs, int obs_cols, const float* critic_obs, int critic_cols, const float* eps,
                           float* mean, float* actions, float* sigma, float* logp, float* value, int batch,
                           void* stream) {
  if (!params || !dims || !frag || !y1 || !obs || !critic_obs || !eps || !mean || !actions || !sigma || !logp ||
      !value || batch < 0)
    return -1;
  if (!ph_dims_match(dims)) return 1;
  if (obs_cols < PH_OBS_SHORT || critic_cols != PH_CRITIC) return 1;
  if (batch == 0) return 0;
  if ((reinterpret_cast<uintptr_t>(frag) & 15u) != 0) return -1;
  PhParams P;
  if (!ph_params(params, P)) return -1;
  const char* hv = getenv("T1POLICY_HEADS64");  // 0: the 32-env k_heads (A/B)
  if (!(hv && hv[0] == '0')) {
    const PhOut64 G{eps, P.std, mean, actions, sigma, logp, value, 0, batch};
    const int tiles = (batch + 63) / 64;
    hipLaunchKernelGGL(k_heads64, dim3(16 * ((tiles + 7) / 8)), dim3(64 * PH_WAVES), 0, (hipStream_t)stream,
                       reinterpret_cast<const h8*>(frag), y1, obs, obs_cols, critic_obs, critic_cols, G, batch);
    return hipGetLastError() == hipSuccess ? 0 : -2;
  }
  PhOut G{eps, P.std, mean, actions, sigma, logp, value, 0, false};
  const int tiles = (batch + PH_M - 1) / PH_M;
  const char* xv = getenv("T1POLICY_HEADS_XCD");
  // T1POLICY_HEADS_XCD (A/B): 2 (default) both roles alternating on every XCD, act() 0.139-0.140 ms; 1 actor on XCDs
  // 0-3 / critic on 4-7, 0.142 (the actor chain is 23% longer, so the actor XCDs finish last); 0 alternating
  // workgroups, 0.140 (profiles/r05hx_act_ab.txt)
  const int xcd_split = xv && xv[0] == '0' ? 0 : (xv && xv[0] == '1' ? 1 : 2);
  const int grid = xcd_split == 2 ? 16 * ((tiles + 7) / 8) : (xcd_split ? 8 * ((tiles + 3) / 4) : 2 * tiles);
  hipLaunchKernelGGL(k_heads, dim3(grid), dim3(64 * PH_WAVES), 0, (hipStream_t)stream, P,
                     reinterpret_cast<const h8*>(frag), y1, obs, obs_cols, critic_obs, critic_cols, G, batch,
                     xcd_split);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
