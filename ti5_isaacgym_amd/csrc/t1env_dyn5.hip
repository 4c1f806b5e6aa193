// t1env_dyn5.hip -- k_dyn5, the env step's main launch with the dynamics on every CU at 8192 envs
// (legged_robot.py:399-434 + Isaac Gym simulate(), and in the fused step post-physics, legged_robot.py:458-506).
//
// k_dyn4 (t1env_dynamics.hip) runs 64 envs per workgroup on four waves (two leg waves, two contact helpers): 4 lanes
// per env, 128 workgroups at 8192 envs -- half the chip, one wave per SIMD, each wave one long dependent chain.
// k_dyn5 gives every env 8 lanes: 32 envs per workgroup, both legs of an env in one wave (lanes 0-31 the left legs,
// 32-63 the right legs of the same 32 envs, so every wave is full and the leg index is a per-lane value), and the
// four waves are four roles of the substep (t1_dyn5.h): W0 core (chain, CRBA, fold-in, elimination, base solve,
// integration), W1 bias (RNEA, PD torques, base block, base-box contacts), W2 terrain contacts of the shank and foot,
// W3 self-contacts.  256 workgroups at 8192 envs: every CU.  Per substep
//     W0: forward chain + CRBA backward pass       | W1 / W2 / W3: their terms from the published state
//     S2 --------------------------------------------------------------------------------------------------
//     W0: fold-in, elimination, base system of the | W1-W3: a slice of the workgroup's own history shift
//         two halves (permlane32), solve, backsub,  |
//         integration, publish the state           |
//     S1 --------------------------------------------------------------------------------------------------
// Two barriers per substep (k_dyn4: three); the two legs' base-block contributions meet by v_permlane32_swap.
//
// The robot model is copied to LDS once per launch: with the leg index per lane, model reads indexed by it are LDS
// reads (two addresses per wave) instead of scalar loads.
//
// The history shift is no longer a set of separate workgroups: each workgroup shifts the 65/2 older frames of its
// OWN 32 rows, a slice per substep on W1-W3 while W0 runs its post-S2 chain (those waves would wait for the next state
// anyway).  The epilogue of the same workgroup then writes the newest frames and zeroes its reset rows itself: no
// cross-workgroup handoff, no sc1 stores, no prelaunched shift at any N.
//
// The fused epilogue (post-physics of the workgroup's 32 envs, t1env_fused.h) runs on all four waves: W0 the rewards
// and the reset rows, W1 the state stores and reset_idx, W2 the privileged frame and last_* rows, W3 the actor frame.
#include <hip/hip_runtime.h>

// -DT1_PHASE_PROF (tools/prof_dynamics_phases.py --kernel 5): lane 0 of every wave accumulates shader-clock deltas
// between T1_PROF_MARK points into per-phase buckets; never part of the product build.
#ifdef T1_PHASE_PROF
constexpr int T1_NPROF5 = 24, T1_PROF_WAVES5 = 4;
__device__ unsigned long long g_t1_prof5[T1_PROF_WAVES5][T1_NPROF5];
__shared__ unsigned long long t1_prof_acc5[T1_PROF_WAVES5][T1_NPROF5 + 1];  // [wave][bucket], last = previous mark
__device__ __forceinline__ unsigned long long t1_stamp5() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
__device__ __forceinline__ void t1_prof_mark5(int i) {
  const int w = threadIdx.x / 64;
  const unsigned long long now = t1_stamp5();
  if ((threadIdx.x & 63) == 0) {
    t1_prof_acc5[w][i] += now - t1_prof_acc5[w][T1_NPROF5];
    t1_prof_acc5[w][T1_NPROF5] = now;
  }
}
__device__ __forceinline__ void t1_prof_begin5() {
  const int w = threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0) {
    for (int i = 0; i < T1_NPROF5; ++i) t1_prof_acc5[w][i] = 0;
    t1_prof_acc5[w][T1_NPROF5] = t1_stamp5();
  }
}
__device__ __forceinline__ void t1_prof_end5() {
  const int w = threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0)
    for (int i = 0; i < T1_NPROF5; ++i) atomicAdd(&g_t1_prof5[w][i], t1_prof_acc5[w][i]);
}
#define T1_PROF_MARK(i) t1_prof_mark5(i)
#define T1_PROF_BEGIN() t1_prof_begin5()
#define T1_PROF_END() t1_prof_end5()
#elif defined(T1_ASM_MARKS)  // ISA analysis build (tools/isa_phases.py): the marks as assembly comments
#define T1_ASM_STR2(x) #x
#define T1_ASM_STR(x) T1_ASM_STR2(x)
#define T1_PROF_MARK(i) asm volatile(";@@MARK " #i "@L" T1_ASM_STR(__LINE__))
#define T1_PROF_BEGIN() asm volatile(";@@MARK begin")
#define T1_PROF_END() asm volatile(";@@MARK end")
#else
#define T1_PROF_BEGIN() ((void)0)
#define T1_PROF_END() ((void)0)
#endif

#include "t1_dyn5.h"
#include "t1env_device.h"
#include "t1env_internal.h"
#include "t1env_postphys.h"
#include "t1env_fused.h"
#include "t1env_roles.h"

using namespace t1;

constexpr int NE5 = 32;        // envs per workgroup
constexpr int D5_BLOCK = 256;  // four waves

constexpr int SH_ROUNDS = 16;  // LDS-DMA staging rounds per shift wave and substep (shift_glds below)
struct ShiftRing { float4 blk[3][SH_ROUNDS][64]; };  // [shift wave][round][lane]

// W1's terms: the bias part of each joint rhs (-S_k . sum_{j>=k} g_j), the leg's total bias, both base-box halves
enum : int { B_RG = 0, B_G = 6, B_AC = 12, B_R = 33, B_N = 39 };

struct Dyn5Lds {  // without the in-workgroup shift's staging (the concurrent shift launch, Dyn5LdsSh below)
  DynModel model;
  Rows4<Q_N> st;         // W0 -> all: substep state
  Rows4<B_N> w1;         // W1 -> W0
  Rows4<XCH> w2[2];      // W2 -> W0: terrain terms of the shank [0], foot [1]
  Rows4<XCH> w3[2];      // W3 -> W0: self-contact terms of the shank, foot
  PdStage<64> pd;        // W1: PD constants and action ring of each lane's leg
  float cap[CAP5_N][64];
  float act[12][NE5];    // the clipped actions (epilogue)
  float epi[EPI_N][NE5];  // staged post-physics inputs (epilogue)
  float fr[FR_N][NE5];   // this step's outputs (epilogue)
  float vis[2][64];      // end-of-step restitution episode of the shank [0] (W2 -> W3's report)
  float vift[64];        // the foot's restitution episode (W0 updates it after S2 from amx; W2 / W3 read it)
  float amx[2][64];      // the fastest approach among the foot points of W2 [0] / W3 [1] this substep
  float rtf[2][3][64];   // the report: terrain forces on the shank [0] / foot [1] (W2)
  float rsf[2][3][64];   // the report: self-contact forces on the shank / foot (W3)
  float vib[64];         // end-of-step episode of the base-box half (W1 -> W3's report)
};
struct Dyn5LdsSh : Dyn5Lds {
  ShiftRing ring;        // the in-workgroup history shift's LDS-DMA staging (W1-W3)
};
template <bool SH> struct Dyn5LdsT { typedef Dyn5Lds type; };
template <> struct Dyn5LdsT<true> { typedef Dyn5LdsSh type; };

__device__ __forceinline__ void read_state(const Dyn5Lds& L, int lane, BaseState<float>& sb, float q[NLEG], float qd[NLEG]) {
  read_state_rows(L.st, lane, sb, q, qd);
}

// ---- the in-workgroup shift staged through LDS by LDS-DMA (global_load_lds, no VGPR destination): the source blocks
// of substep s's slice are loaded at the end of substep s-1's post-S2 window (in the prologue for s = 0) and land while
// the waves run their substep-s role work; after S2 of substep s each wave forms its outputs from its own staged blocks
// (ds_read) and stores them, then issues the loads of slice s + 1.  A wave-round loads 64 consecutive 16-B blocks of
// the input (one per lane) and writes 63 output chunks (chunk c reads its source from the blocks c + F/per and
// c + F/per + 1), so a wave reads only blocks it loaded itself and needs no barrier between DMA and use (its own
// vmcnt); rounds go round-robin over the three shift waves.  32-row workgroups need at most 15 rounds per wave and
// substep (fp32: 14 of the 66-frame history + 1 of the critic's).
constexpr int SH_OUT = 63;                   // output chunks per round
typedef __attribute__((address_space(3))) void* t1_lds_vp;
// One LDS-DMA of 16 B per lane into the wave-uniform LDS address lds_dst (+ lane x 16), by inline assembly: hipcc does
// not count an asm load, so it adds no vmcnt(0) before the later LDS reads of other data (with the builtin it waited
// for every outstanding store before each ring read, which serialised the shift on store acknowledgements); the ring is
// instead retired by an explicit vmcnt(0) before the S2 barrier (shift_glds_retire).  M0 is saved and restored in the
// statement (cdna_hip_programming.md, LDS-DMA recipe).
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  unsigned keep;
  // nt: the shift's streaming loads (and stores, shift_glds_out) non-temporal, sparing the L2 for the terrain's
  // height samples (-2.7% step time with the speculative terrain queries, r04i)
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}
__device__ __forceinline__ void shift_glds_retire() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

template <int F, int H, bool HALF> struct ShiftHist {
  static constexpr uint32_t ROW = F * H, PER = HALF ? 8 : 4, ES = HALF ? 2 : 4, D = F / PER, REM = F % PER;
};
// output chunks of the workgroup's rows of one history (16-B chunks), and the elements from the rows' start to the
// buffer end
template <int F, int H, bool HALF>
__device__ __forceinline__ void shift_extent(int64_t total, int64_t r0, int64_t r1, uint32_t& n_out, uint32_t& lim) {
  using SH = ShiftHist<F, H, HALF>;
  lim = (uint32_t)(total - r0 * (int64_t)SH::ROW);
  const uint32_t span = (uint32_t)((r1 - r0) * SH::ROW);
  n_out = ((span < lim ? span : lim) + SH::PER - 1) / SH::PER;
}
// issue the DMA of this wave's rounds of the slice [c_lo, c_hi) into ring rounds [slot0, ...); returns the rounds used
template <int F, int H, bool HALF>
__device__ __forceinline__ int shift_glds_issue(const void* in, int64_t total, int64_t r0, int64_t r1, uint32_t c_lo,
                                               uint32_t c_hi, int w, int lane, ShiftRing& R, int slot0) {
  using SH = ShiftHist<F, H, HALF>;
  uint32_t n_out, lim;
  shift_extent<F, H, HALF>(total, r0, r1, n_out, lim);
  const uint32_t hi = c_hi < n_out ? c_hi : n_out;
  if (hi <= c_lo || lim < 2 * SH::PER) return 0;
  const int rounds = (int)((hi - c_lo + SH_OUT - 1) / SH_OUT);
  const uint8_t* in0 = reinterpret_cast<const uint8_t*>(in) + (size_t)(r0 * SH::ROW) * SH::ES;
  const uint32_t last = lim / SH::PER - 1;  // the last whole block in the buffer
  int j = 0;
  for (int k = w; k < rounds; k += 3, ++j) {
    uint32_t b = c_lo + (uint32_t)k * SH_OUT + SH::D + (uint32_t)lane;
    b = b < last ? b : last;  // past the buffer end: a valid dummy block (its outputs are not stored)
    glds16(in0 + (size_t)b * 16, (uint32_t)(size_t)(t1_lds_vp)&R.blk[w][slot0 + j][0]);
  }
  return j;
}
// one output chunk c (16 B) from the two staged source blocks xa, xb; TAIL: the second block may pass the buffer end
// (the buffer's last rows), the source is then read from global memory element by element
template <int F, int H, bool HALF, bool TAIL>
__device__ __forceinline__ void shift_glds_out(const void* in, void* out, int64_t r0, uint32_t lim, uint32_t c, float4 xa,
                                               float4 xb) {
  using SH = ShiftHist<F, H, HALF>;
  const uint32_t i = c * SH::PER;  // first output element (rows-relative)
  const uint32_t col0 = i - (i / SH::ROW) * SH::ROW;
  if constexpr (!HALF) {
    const float* in0 = reinterpret_cast<const float*>(in) + r0 * SH::ROW;
    float* out0 = reinterpret_cast<float*>(out) + r0 * SH::ROW;
    float src[8] = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w};
    if constexpr (TAIL) {
#pragma unroll
      for (int k2 = 0; k2 < 8; ++k2) {
        const uint32_t e = (c + SH::D) * 4 + k2;
        src[k2] = e < lim ? in0[e] : 0.0f;
      }
    }
    if (col0 + 3 < SH::ROW - F && i + 3 < lim) {
      const float4 o4 = make_float4(src[SH::REM], src[SH::REM + 1], src[SH::REM + 2], src[SH::REM + 3]);
      typedef float f4v __attribute__((ext_vector_type(4)));
      __builtin_nontemporal_store(f4v{o4.x, o4.y, o4.z, o4.w}, reinterpret_cast<f4v*>(out0 + i));
      return;
    }
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2) {
      const uint32_t e = i + k2;
      if (e >= lim) break;
      if (e - (e / SH::ROW) * SH::ROW < SH::ROW - F) out0[e] = src[SH::REM + k2];
    }
  } else {
    constexpr uint32_t MM = SH::REM / 2;
    const uint16_t* in0 = reinterpret_cast<const uint16_t*>(in) + r0 * SH::ROW;
    uint16_t* out0 = reinterpret_cast<uint16_t*>(out) + r0 * SH::ROW;
    const u32x4 a = __builtin_bit_cast(u32x4, xa), b = __builtin_bit_cast(u32x4, xb);
    uint32_t wv[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    if constexpr (TAIL) {
#pragma unroll
      for (int k2 = 0; k2 < 8; ++k2) {
        const uint32_t e = (c + SH::D) * 8 + 2 * k2;
        const uint32_t lo = e < lim ? in0[e] : 0u, hh = e + 1 < lim ? in0[e + 1] : 0u;
        wv[k2] = lo | (hh << 16);
      }
    }
    u32x4 o;
    if constexpr (SH::REM % 2 == 0) {
      o = u32x4{wv[MM], wv[MM + 1], wv[MM + 2], wv[MM + 3]};
    } else {
      o = u32x4{__builtin_amdgcn_alignbyte(wv[MM + 1], wv[MM], 2), __builtin_amdgcn_alignbyte(wv[MM + 2], wv[MM + 1], 2),
                __builtin_amdgcn_alignbyte(wv[MM + 3], wv[MM + 2], 2), __builtin_amdgcn_alignbyte(wv[MM + 4], wv[MM + 3], 2)};
    }
    if (col0 + 7 < SH::ROW - F && i + 7 < lim) {
      __builtin_nontemporal_store(o, reinterpret_cast<u32x4*>(out0 + i));
      return;
    }
    const uint32_t ow[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2) {
      const uint32_t e = i + k2;
      if (e >= lim) break;
      if (e - (e / SH::ROW) * SH::ROW < SH::ROW - F) out0[e] = (uint16_t)(ow[k2 / 2] >> (16 * (k2 & 1)));
    }
  }
}
// form and store this wave's outputs of the slice [c_lo, c_hi) from its staged rounds (their DMA retired)
template <int F, int H, bool HALF>
__device__ __forceinline__ int shift_glds_commit(const void* in, void* out, int64_t total, int64_t r0, int64_t r1,
                                                uint32_t c_lo, uint32_t c_hi, int w, int lane, const ShiftRing& R,
                                                int slot0) {
  using SH = ShiftHist<F, H, HALF>;
  uint32_t n_out, lim;
  shift_extent<F, H, HALF>(total, r0, r1, n_out, lim);
  const uint32_t hi = c_hi < n_out ? c_hi : n_out;
  if (hi <= c_lo || lim < 2 * SH::PER) return 0;
  const int rounds = (int)((hi - c_lo + SH_OUT - 1) / SH_OUT);
  // chunks whose second source block would pass the buffer end (the buffer's last rows) take the TAIL form
  const uint32_t c_tail = lim / SH::PER >= SH::D + 2 ? lim / SH::PER - SH::D - 1 : 0u;
  const bool any_tail = hi > c_tail;  // wave-uniform
  int j = 0;
  for (int k = w; k < rounds; k += 3, ++j) {
    const uint32_t c = c_lo + (uint32_t)k * SH_OUT + (uint32_t)lane;
    const float4 xa = R.blk[w][slot0 + j][lane];
    const float4 xb = R.blk[w][slot0 + j][lane < 63 ? lane + 1 : 63];
    if (lane >= SH_OUT || c >= hi) continue;
    if (!any_tail) shift_glds_out<F, H, HALF, false>(in, out, r0, lim, c, xa, xb);
    else if (c < c_tail) shift_glds_out<F, H, HALF, false>(in, out, r0, lim, c, xa, xb);
    else shift_glds_out<F, H, HALF, true>(in, out, r0, lim, c, xa, xb);
  }
  return j;
}
// slice `sl` of `nsl` of both histories: issue its DMA / commit its outputs (shift wave w of 3)
template <bool HALF>
__device__ __forceinline__ void shift_glds_slice(const ShiftArgs& S, int64_t r0, int64_t r1, int sl, int nsl, int w,
                                                 int lane, ShiftRing& R, bool commit) {
  if (r1 <= r0 || sl >= nsl) return;
  uint32_t no, np, lim;
  shift_extent<T1_NOBS, T1_HIST, HALF>(S.total_obs, r0, r1, no, lim);
  shift_extent<T1_NPRIV, T1_CHIST, HALF>(S.total_priv, r0, r1, np, lim);
  const uint32_t olo = no * sl / nsl, ohi = no * (sl + 1) / nsl, plo = np * sl / nsl, phi = np * (sl + 1) / nsl;
  if (commit) {
    const int used = shift_glds_commit<T1_NOBS, T1_HIST, HALF>(S.obs_in, S.obs_out, S.total_obs, r0, r1, olo, ohi, w,
                                                               lane, R, 0);
    shift_glds_commit<T1_NPRIV, T1_CHIST, HALF>(S.priv_in, S.priv_out, S.total_priv, r0, r1, plo, phi, w, lane, R, used);
  } else {
    const int used = shift_glds_issue<T1_NOBS, T1_HIST, HALF>(S.obs_in, S.total_obs, r0, r1, olo, ohi, w, lane, R, 0);
    shift_glds_issue<T1_NPRIV, T1_CHIST, HALF>(S.priv_in, S.total_priv, r0, r1, plo, phi, w, lane, R, used);
  }
}
__device__ __forceinline__ void shift_glds(const ShiftArgs& S, int64_t r0, int64_t r1, int sl, int nsl, int w, int lane,
                                           ShiftRing& R, bool commit) {
#ifdef T1_WHATIF_D5_NO_SHIFT  // timing-only what-if build: the history is not shifted
  return;
#endif
  if (S.half) shift_glds_slice<true>(S, r0, r1, sl, nsl, w, lane, R, commit);
  else shift_glds_slice<false>(S, r0, r1, sl, nsl, w, lane, R, commit);
}

// ---------------------------------------------------------------------------------------------------
// k_dyn5.  Lane l of every wave: env blockIdx.x * 32 + (l & 31), leg l >> 5.  Inactive lanes (past num_envs) shadow
// the last env and store nothing.  The substep log (tests only, LG.root != nullptr) is a run-time switch of the one
// product code object, like k_dyn4's.
// ---------------------------------------------------------------------------------------------------
template <bool HF, bool FUSED, bool SH>
__global__ __launch_bounds__(D5_BLOCK) void k_dyn5(const DynModel* __restrict__ Mg, const t1env_config* __restrict__ Cp,
                                                   t1env_buffers B, Terrain Tin, const float* __restrict__ actions,
                                                   t1env_step_args A, ShiftArgs S, int dyn_blocks, FusedArgs FA,
                                                   SubLog LG) {
  __shared__ typename Dyn5LdsT<SH>::type lds;
  {  // the model to LDS
    constexpr int NW = (int)(sizeof(DynModel) / 4);
    static_assert(sizeof(DynModel) % 4 == 0, "the model copies as words");
    const uint32_t* src = reinterpret_cast<const uint32_t*>(Mg);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&lds.model);
    for (int i = threadIdx.x; i < NW; i += D5_BLOCK) dst[i] = src[i];
  }
  Terrain T = Tin;
  T.type = HF ? 2 : 0;
  const t1env_config& C = *Cp;
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x / 64);
  const int lane = threadIdx.x & 63;
#ifdef T1_WHATIF_D5_SCALAR_MODEL  // timing-only what-if: every lane runs the left leg's model through scalar loads
  const int leg = 0;
#else
  const int leg = lane >> 5;
#endif
  const int e = lane & 31;
  const int j0 = 6 * leg;
  const int N = C.num_envs;
  const int n0 = (int)blockIdx.x * NE5 + e;
  const bool active = n0 < N;
  const int n = active ? n0 : N - 1;
  const float dt = C.sim_dt;
  const uint32_t ctr = A.counter;
  const int nsub = C.decimation;
  const int64_t r0 = (int64_t)blockIdx.x * NE5, r1 = r0 + NE5 < N ? r0 + NE5 : N;
  T1_PROF_BEGIN();
  __syncthreads();  // the model in LDS
#ifdef T1_WHATIF_D5_SCALAR_MODEL
  const DynModel& M = *Mg;
#else
  const DynModel& M = lds.model;
#endif

  if (wave == 1) {
    // ---------------- W1: RNEA bias terms of the leg, both base-box halves
    BaseParams<float> PB;
    LegParams<float> PL;
    load_base_params(M, B, n, PB);
    load_leg_params(M, B, n, j0, PL);
    const float mu = PB.friction, eg = ground_restitution(M, PB.restitution);
    float vi_b = B.contact_vimp[(size_t)n * NVIMP + vimp_base(leg)];
    int cb, ce;
    base_contact_range(M, leg, cb, ce);
    const float zero6[NLEG] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    if constexpr (SH) shift_glds(S, r0, r1, 0, nsub, 0, lane, lds.ring, false);  // the first slice's DMA
    T1_PROF_MARK(0);
    for (int sub = 0; sub < nsub; ++sub) {
      __syncthreads();  // S1: the substep state published
      T1_PROF_MARK(1);
      BaseState<float> sb;
      float q[NLEG], qd[NLEG];
      read_state(lds, lane, sb, q, qd);
      BaseFrame<float> F;
      base_frame(sb, F);
      const int32_t bound_b = terrain_bound_raw_any(T, F.abs.x, F.abs.y);
      // the base box half's queries issued before the bound is tested (see body_contact_fixed_q), under the bias pass
      ContactQuery<T1_POINTS_PER_BODY / 2, float> Qb;
      contact_query<HF, T1_POINTS_PER_BODY / 2>(M, T, cb, F.R0, v3<float>(0, 0, 0), F.abs, Qb);
      T1_PROF_MARK(2);
      float v[B_N];
      {
        float rg[NLEG], G[6];
        leg_bias_rhs(M, PL, F, q, qd, zero6, leg, dt, rg, G);  // -S_k . sum g (W0 adds dt tau_k)
#pragma unroll
        for (int k = 0; k < NLEG; ++k) v[B_RG + k] = rg[k];
#pragma unroll
        for (int i = 0; i < 6; ++i) v[B_G + i] = G[i];
      }
      T1_PROF_MARK(3);
      {  // the base-box halves, summed left first (the same sum in both halves)
        Sym6<float> Cb;
        float gw[6] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
        sym_zero(Cb);
        body_contact_fixed_q<HF, T1_POINTS_PER_BODY / 2>(M, Qb, F.abs.z - M.contact_radius[0], bound_b, T, F.V0, mu,
                                                         eg, vi_b, dt, Cb, gw);
#pragma unroll
        for (int i = 0; i < 21; ++i) {
          float l, rr;
          halves(Cb.a[i], l, rr);
          v[B_AC + i] = l + rr;
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          float l, rr;
          halves(gw[i], l, rr);
          v[B_R + i] = -l - rr;
        }
      }
      T1_PROF_MARK(4);
      put4(lds.w1, lane, v);
      if constexpr (SH) shift_glds_retire();  // this substep's staged slice landed (issued a substep ago) before S2
      T1_PROF_MARK(5);
      __syncthreads();  // S2: the terms published
      T1_PROF_MARK(6);
      if constexpr (SH) {
        // this substep's staged slice (its DMA retired before S2), then the next slice's DMA
        shift_glds(S, r0, r1, sub, nsub, wave - 1, lane, lds.ring, true);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the ring reads done before the DMA rewrites it
        shift_glds(S, r0, r1, sub + 1, nsub, wave - 1, lane, lds.ring, false);
      }
      T1_PROF_MARK(7);
    }
    lds.vib[lane] = vi_b;
    if (active) B.contact_vimp[(size_t)n * NVIMP + vimp_base(leg)] = vi_b;
    if constexpr (SH) __builtin_amdgcn_s_waitcnt(0);  // the shift's stores complete before the epilogue zeroes reset rows
    __syncthreads();  // R1: the end-of-step state and episodes published
    T1_PROF_MARK(9);
    {  // the report's base-box force (leg-0 lanes: the whole box, the larger restitution set point of its halves)
      V3<float> fb = v3<float>(0.0f, 0.0f, 0.0f);
      if (leg == 0) {
        BaseState<float> sb;
        float q[NLEG], qd[NLEG];
        read_state(lds, lane, sb, q, qd);
        BaseFrame<float> F;
        base_frame(sb, F);
        const float vt0 = restitution_target(M, eg, lds.vib[lane]), vt1 = restitution_target(M, eg, lds.vib[lane ^ 32]);
        fb = body_contact_force(M, T, 0, F.R0, v3<float>(0, 0, 0), F.abs, F.V0, mu, vt0 > vt1 ? vt0 : vt1);
      }
      T1_PROF_MARK(10);
      __syncthreads();  // RB: the report's parts in LDS
      if (leg == 0) {
        if (active) {
          float* cf = B.contact_forces + (size_t)n * 39;
          cf[0] = fb.x; cf[1] = fb.y; cf[2] = fb.z;
        }
        if constexpr (FUSED) { lds.fr[F_CFB][e] = fb.x; lds.fr[F_CFB + 1][e] = fb.y; lds.fr[F_CFB + 2][e] = fb.z; }
      }
    }
    if constexpr (FUSED) {
      __syncthreads();  // the epilogue barrier
      T1_PROF_MARK(11);
      fused_epilogue_staged<POST_A_STATE, NE5, SH>(M, C, B, A, S, FA, dyn_blocks, lane, lds.epi, lds.fr, lds.act,
                                                     lds.act + NLEG);
    }
    T1_PROF_END();
    return;
  }

  if (wave >= 2) {
    // ---------------- W2: shank terrain + foot points 0-3 / W3: self-contacts + foot points 4-7
    const float mu = 0.5f * (B.friction[n] + M.ground_friction);  // robot shape vs ground (PhysX average)
    const float mu_self = B.friction[n];                          // robot shape vs robot shape
    const float eg = ground_restitution(M, B.restitution[n]);
    float vi_sh = wave == 2 ? B.contact_vimp[(size_t)n * NVIMP + vimp_shank(leg)] : 0.0f;
    // the epilogue's inputs the step does not change, staged while W0 sets up (nothing writes them before the epilogue)
    if constexpr (FUSED) stage_epilogue_inputs<NE5, 128>(B, N, (int)r0, (int)threadIdx.x - 128, lds.epi);
    const int bsh = 1 + 6 * leg + K_SHANK, bft = 1 + 6 * leg + K_FOOT;
    const int foot_c0 = M.contact_start[bft] + (wave == 2 ? 0 : T1_POINTS_PER_BODY / 2);
    if constexpr (SH) shift_glds(S, r0, r1, 0, nsub, wave - 1, lane, lds.ring, false);  // the first slice's DMA
    T1_PROF_MARK(0);
    for (int sub = 0; sub < nsub; ++sub) {
      __syncthreads();  // S1
      T1_PROF_MARK(1);
      BaseState<float> sb;
      float q[NLEG], qd[NLEG];
      read_state(lds, lane, sb, q, qd);
      BaseFrame<float> F;
      base_frame(sb, F);
      BodyKin<float> Ko[2];
      leg_body_kinematics(M, F, q, qd, leg, Ko);
      const float vtg_ft = restitution_target(M, eg, lds.vift[lane]);  // this substep's foot episode (W0 keeps it)
      T1_PROF_MARK(2);
      Sym6<float> Cs[2];
      float cs[2][6];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        sym_zero(Cs[i]);
#pragma unroll
        for (int j = 0; j < 6; ++j) cs[i][j] = 0.0f;
      }
      // this wave's half of the foot's points: queries first, their heights used after the wave's other work
      ContactQuery<T1_POINTS_PER_BODY / 2, float> Qf;
      contact_query<HF, T1_POINTS_PER_BODY / 2>(M, T, foot_c0, Ko[1].Rb, Ko[1].p, F.abs, Qf);
      if (wave == 2) {
        // the shank's queries issued with the foot's and the bound's, before the bound is tested (one memory round
        // trip instead of two)
        ContactQuery<T1_POINTS_PER_BODY, float> Qs;
        contact_query<HF, T1_POINTS_PER_BODY>(M, T, M.contact_start[bsh], Ko[0].Rb, Ko[0].p, F.abs, Qs);
        const int32_t bnd = terrain_bound_raw_any(T, Ko[0].p.x + F.abs.x, Ko[0].p.y + F.abs.y);
        body_contact_fixed_q<HF, T1_POINTS_PER_BODY>(M, Qs, Ko[0].p.z + F.abs.z - M.contact_radius[bsh], bnd, T,
                                                     Ko[0].V, mu, eg, vi_sh, dt, Cs[0], cs[0]);
      } else if (M.self_collisions) {
        SelfBody<float> O[2], X[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          O[s] = self_body(M, leg, s, Ko[s]);
          const float mine[12] = {O[s].cap.p.x, O[s].cap.p.y, O[s].cap.p.z, O[s].cap.q.x, O[s].cap.q.y,
                                  O[s].cap.q.z, O[s].V[0],    O[s].V[1],    O[s].V[2],    O[s].V[3],
                                  O[s].V[4],    O[s].V[5]};
          float oth[12];
#pragma unroll
          for (int i = 0; i < 12; ++i) {
            float l, r;
            halves(mine[i], l, r);
            oth[i] = leg ? l : r;
          }
          X[s].cap.p = v3<float>(oth[0], oth[1], oth[2]);
          X[s].cap.q = v3<float>(oth[3], oth[4], oth[5]);
          X[s].cap.r = M.self_cap[1 - leg][s].r;
#pragma unroll
          for (int i = 0; i < 6; ++i) X[s].V[i] = oth[6 + i];
        }
        self_terms_bodies(M, leg, O, X, mu_self, dt, Cs, cs);
      }
      T1_PROF_MARK(3);
      float amax = -1.0f;
      if (t1_wave_any(vtg_ft > 0.0f))
        contact_apply<HF, T1_POINTS_PER_BODY / 2>(M, Qf, Ko[1].V, mu, vtg_ft, dt, Cs[1], cs[1], amax);
      else
        contact_apply<HF, T1_POINTS_PER_BODY / 2>(M, Qf, Ko[1].V, mu, 0.0f, dt, Cs[1], cs[1], amax);
      T1_PROF_MARK(4);
      {
        Rows4<XCH>* dst = wave == 2 ? lds.w2 : lds.w3;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          float v[XCH];
          sym_pack(Cs[i], cs[i], v);
          put4(dst[i], lane, v);
        }
        lds.amx[wave - 2][lane] = amax;
      }
      if constexpr (SH) shift_glds_retire();  // this substep's staged slice landed (issued a substep ago) before S2
      T1_PROF_MARK(5);
      __syncthreads();  // S2
      T1_PROF_MARK(6);
      if constexpr (SH) {
        // this substep's staged slice (its DMA retired before S2), then the next slice's DMA
        shift_glds(S, r0, r1, sub, nsub, wave - 1, lane, lds.ring, true);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the ring reads done before the DMA rewrites it
        shift_glds(S, r0, r1, sub + 1, nsub, wave - 1, lane, lds.ring, false);
      }
      T1_PROF_MARK(7);
    }
    if (wave == 2) {
      lds.vis[0][lane] = vi_sh;
      if (active) B.contact_vimp[(size_t)n * NVIMP + vimp_shank(leg)] = vi_sh;
    }
    if constexpr (SH) __builtin_amdgcn_s_waitcnt(0);  // the shift's stores complete before the epilogue zeroes reset rows
    __syncthreads();  // R1: the end-of-step state and episodes published
    T1_PROF_MARK(9);
    {  // the contact-force report from the end-of-step state: W2 the terrain forces of its leg's shank and foot, W3
       // their self-contact forces; W2 sums them after RB (the base box: W1)
      BaseState<float> sb;
      float q[NLEG], qd[NLEG];
      read_state(lds, lane, sb, q, qd);
      BaseFrame<float> F;
      base_frame(sb, F);
      BodyKin<float> Ko[2];
      leg_body_kinematics(M, F, q, qd, leg, Ko);
      if (wave == 2) {
        const float vt[2] = {restitution_target(M, eg, lds.vis[0][lane]), restitution_target(M, eg, lds.vift[lane])};
#pragma unroll
        for (int sb2 = 0; sb2 < 2; ++sb2) {
          const int b = 1 + 6 * leg + (sb2 == 0 ? K_SHANK : K_FOOT);
          const V3<float> f = body_contact_force(M, T, b, Ko[sb2].Rb, Ko[sb2].p, F.abs, Ko[sb2].V, mu, vt[sb2]);
          lds.rtf[sb2][0][lane] = f.x; lds.rtf[sb2][1][lane] = f.y; lds.rtf[sb2][2][lane] = f.z;
        }
      } else {
        V3<float> fself[2] = {v3<float>(0.0f, 0.0f, 0.0f), v3<float>(0.0f, 0.0f, 0.0f)};
        if (M.self_collisions) {
          SelfBody<float> O[2], X[2];
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            O[s] = self_body(M, leg, s, Ko[s]);
            const float mine[12] = {O[s].cap.p.x, O[s].cap.p.y, O[s].cap.p.z, O[s].cap.q.x, O[s].cap.q.y, O[s].cap.q.z,
                                    O[s].V[0],    O[s].V[1],    O[s].V[2],    O[s].V[3],    O[s].V[4],    O[s].V[5]};
            float oth[12];
#pragma unroll
            for (int i = 0; i < 12; ++i) {
              float l, r;
              halves(mine[i], l, r);
              oth[i] = leg ? l : r;
            }
            X[s].cap.p = v3<float>(oth[0], oth[1], oth[2]);
            X[s].cap.q = v3<float>(oth[3], oth[4], oth[5]);
            X[s].cap.r = M.self_cap[1 - leg][s].r;
#pragma unroll
            for (int i = 0; i < 6; ++i) X[s].V[i] = oth[6 + i];
          }
          self_forces_bodies(M, leg, O, X, mu_self, fself);
        }
#pragma unroll
        for (int sb2 = 0; sb2 < 2; ++sb2) {
          lds.rsf[sb2][0][lane] = fself[sb2].x; lds.rsf[sb2][1][lane] = fself[sb2].y; lds.rsf[sb2][2][lane] = fself[sb2].z;
        }
      }
      T1_PROF_MARK(10);
      __syncthreads();  // RB: the report's parts in LDS
      if (wave == 2) {
        float* cf = B.contact_forces + (size_t)n * 39;
#pragma unroll
        for (int sb2 = 0; sb2 < 2; ++sb2) {
          const int b = 1 + 6 * leg + (sb2 == 0 ? K_SHANK : K_FOOT);
          const float f[3] = {lds.rtf[sb2][0][lane] + lds.rsf[sb2][0][lane], lds.rtf[sb2][1][lane] + lds.rsf[sb2][1][lane],
                              lds.rtf[sb2][2][lane] + lds.rsf[sb2][2][lane]};
          if (active) { cf[b * 3 + 0] = f[0]; cf[b * 3 + 1] = f[1]; cf[b * 3 + 2] = f[2]; }
          if (FUSED && sb2 == 1) {
            const int r = leg == 0 ? F_C0 : F_C1;
            lds.fr[r][e] = f[0]; lds.fr[r + 1][e] = f[1]; lds.fr[r + 2][e] = f[2];
          }
        }
      }
    }
    if constexpr (FUSED) {
      __syncthreads();  // the epilogue barrier
      T1_PROF_MARK(11);
      if (wave == 2)
        fused_epilogue_obs<POST_OBS_PRIV, NE5>(M, C, B, A, lane, lds.epi, lds.fr, lds.act, lds.act + NLEG);
      else
        fused_epilogue_obs<POST_OBS_ACTOR, NE5>(M, C, B, A, lane, lds.epi, lds.fr, lds.act, lds.act + NLEG);
      T1_PROF_MARK(15);
    }
    T1_PROF_END();
    return;
  }

  // ---------------- W0: core -- PD torques, base block, chain + CRBA; after S2 fold-in, elimination, base system,
  // integration; owns the actions, the PD staging and the foot's restitution episode
  BaseParams<float> PB;
  LegParams<float> PL;
  BaseState<float> sb;
  float q[NLEG], qd[NLEG];
  load_base_params(M, B, n, PB);
  load_leg_params(M, B, n, j0, PL);
  load_base_state(M, PB, B.root_states + (size_t)n * 13, sb);
#pragma unroll
  for (int k = 0; k < NLEG; ++k) {
    q[k] = B.dof_state[n * 24 + 2 * (j0 + k)];
    qd[k] = B.dof_state[n * 24 + 2 * (j0 + k) + 1];
  }
  // every per-env load of the prologue is issued before its first global store (the buffers may alias as far as the
  // compiler knows, so a load after a store would cost another memory round trip)
  const int lag = B.lag_timestep[n];
  const RngKey K = rng_key(C.seed, (uint32_t)(C.env_offset + n), ctr);
  const V3<float> ef = v3<float>(B.applied_force[n * 3 + 0], B.applied_force[n * 3 + 1], B.applied_force[n * 3 + 2]);
  float vi_ft = B.contact_vimp[(size_t)n * NVIMP + vimp_foot(leg)];
  int s_dof = 9 - B.dof_lag_timestep[n] % 10;
#ifdef T1_MUTANT_CAPTURE  // mutation check of tests/test_gpu_product_parity.py only (tools/gpu): capture a substep early
  s_dof = s_dof > 0 ? s_dof - 1 : 0;
#endif
  const int s_imu = 9 - B.imu_lag_timestep[n] % 10;
  {  // actions = clip(actions) into the step's history slot, the PD constants and action ring staged
    PdStage<64>& P = lds.pd;
    float a[NLEG];
#pragma unroll
    for (int k = 0; k < NLEG; ++k) a[k] = fminf(fmaxf(actions[n * 12 + j0 + k], -C.clip_actions), C.clip_actions);
    const int cs = (int)(ctr & 3u);
#pragma unroll
    for (int k = 0; k < NLEG; ++k) {
      const int j = j0 + k;
      P.kp[k][lane] = B.kp[n * 12 + j];
      P.kd[k][lane] = B.kd[n * 12 + j];
      P.off[k][lane] = B.motor_offsets[n * 12 + j];
      P.visc[k][lane] = B.viscous[n * 12 + j];
      P.coul[k][lane] = B.coulomb[n * 12 + j];
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int k = 0; k < NLEG; ++k)
        P.act[s][k][lane] = s == cs ? a[k] * C.action_scale : B.act_hist[((size_t)n * 4 + s) * 12 + j0 + k];
#pragma unroll
    for (int k = 0; k < NLEG; ++k) lds.act[j0 + k][e] = a[k];
    if (active) {
      float* slot = B.act_hist + ((size_t)n * 4 + cs) * 12;
#pragma unroll
      for (int k = 0; k < NLEG; ++k) {
        B.actions[n * 12 + j0 + k] = a[k];
        slot[j0 + k] = a[k] * C.action_scale;
      }
    }
  }
  lds.vift[lane] = vi_ft;
  float* const dof_dst = B.dof_hist + ((size_t)n * 4 + (ctr & 3u)) * 24;
  float* const imu_dst = B.imu_hist + ((size_t)n * 2 + (ctr & 1u)) * 8;
  float tau[NLEG];
  {
    float v[Q_N];
    state_pack(sb, q, qd, v);
    put4(lds.st, lane, v);
  }
  T1_PROF_MARK(0);
  for (int sub = 0; sub < nsub; ++sub) {
    __syncthreads();  // S1: the substep state published
    T1_PROF_MARK(1);
    BaseFrame<float> F;
    base_frame(sb, F);
    pd_torques_staged(M, C, lds.pd, lane, K, ctr, sub, lag, j0, q, qd, tau);
    Sym6<float> Ac;  // the base body's block (both halves compute it: the same values)
    float r[6];
    base_block(M, PB, F, sub == 0 ? ef : v3<float>(0, 0, 0), dt, Ac, r);
    LegFK<float> fk;
    leg_fk_chain(M, F.R0, q, leg, fk);
    T1_PROF_MARK(2);
    float Sj[NLEG][6];
    LegBlock<float> lb;
    Sym6<float> Ab;
    sym_zero(Ab);
    leg_backward_crba(M, PL, q, qd, leg, dt, fk, Sj, lb, Ab);
    T1_PROF_MARK(3);
    __syncthreads();  // S2: W1-W3's terms published
    T1_PROF_MARK(4);
    float g6[6] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    float w1v[B_N];
    get4(lds.w1, lane, w1v);
    {  // the foot's episode from the two halves of its points
      const float am = fmaxf(lds.amx[0][lane], lds.amx[1][lane]);
      vi_ft = restitution_episode(vi_ft, am);
      lds.vift[lane] = vi_ft;  // W2 / W3 read it after the next S1
    }
    {
      float rg[NLEG], G[6];
#pragma unroll
      for (int k = 0; k < NLEG; ++k) rg[k] = dt * tau[k] + w1v[B_RG + k];
#pragma unroll
      for (int i = 0; i < 6; ++i) G[i] = w1v[B_G + i];
      Sym6<float> Cb[2];
      float cb[2][6];
#pragma unroll
      for (int i = 0; i < 2; ++i) {  // shank [0]: W2 terrain + W3 self; foot [1]: W2 half + W3 self and half
        float vt[XCH], vs[XCH];
        get4(lds.w2[i], lane, vt);
        get4(lds.w3[i], lane, vs);
#pragma unroll
        for (int k = 0; k < XCH; ++k) vt[k] += vs[k];
        sym_unpack(vt, Cb[i], cb[i]);
      }
      leg_apply_terms<K_SHANK, K_FOOT>(Cb[0], cb[0], Cb[1], cb[1], rg, G, Sj, lb, Ab, g6);
    }
    T1_PROF_MARK(5);
    float rb[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) rb[i] = -g6[i];
    eliminate_leg(lb, Ab, rb);
    T1_PROF_MARK(6);
    // the base system: (base block + both base-box halves) + the left leg + the right leg, in every lane
#pragma unroll
    for (int i = 0; i < 21; ++i) {
      float l, rr;
      halves(Ab.a[i], l, rr);
      Ac.a[i] = ((Ac.a[i] + w1v[B_AC + i]) + l) + rr;
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      float l, rr;
      halves(rb[i], l, rr);
      r[i] = ((-r[i] + w1v[B_R + i]) + l) + rr;
    }
    solve_base(Ac, r);
    float dq[NLEG];
    backsub_leg(lb, r, dq);
    integrate_base(sb, r, dt);
    integrate_leg(M, leg, q, qd, dq, dt);
    T1_PROF_MARK(7);
    if (LG.root != nullptr) {  // wave-uniform (a kernel argument)
      if (active) {
        const size_t row = (size_t)sub * N + n;
#pragma unroll
        for (int k = 0; k < NLEG; ++k) {
          LG.torque[row * 12 + j0 + k] = tau[k];
          LG.dof[row * 24 + 2 * (j0 + k)] = q[k];
          LG.dof[row * 24 + 2 * (j0 + k) + 1] = qd[k];
        }
        if (leg == 0) {
          BaseFrame<float> FL;
          base_frame(sb, FL);
          float body[13];
          root_row(M, PB, sb, FL, body);
#pragma unroll
          for (int i = 0; i < 13; ++i) LG.root[row * 13 + i] = body[i];
        }
      }
    }
    if (sub == s_dof) {
#pragma unroll
      for (int k = 0; k < NLEG; ++k) { lds.cap[k][lane] = q[k]; lds.cap[NLEG + k][lane] = qd[k]; }
    }
    if (leg == 0 && sub == s_imu) {
#pragma unroll
      for (int i = 0; i < 4; ++i) lds.cap[2 * NLEG + i][lane] = sb.quat[i];
#pragma unroll
      for (int i = 0; i < 3; ++i) lds.cap[2 * NLEG + 4 + i][lane] = sb.w[i];
    }
    float v[Q_N];
    state_pack(sb, q, qd, v);
    put4(lds.st, lane, v);  // W1-W3 read the previous state before S2; after the last substep: the report's
    T1_PROF_MARK(8);
  }
  if (active) {
    B.contact_vimp[(size_t)n * NVIMP + vimp_foot(leg)] = vi_ft;
    if (s_dof < nsub) {  // the sensor-lag samples captured in the loop
#pragma unroll
      for (int k = 0; k < NLEG; ++k) { dof_dst[j0 + k] = lds.cap[k][lane]; dof_dst[12 + j0 + k] = lds.cap[NLEG + k][lane]; }
    }
    if (leg == 0 && s_imu < nsub) {
      const float quat[4] = {lds.cap[2 * NLEG][lane], lds.cap[2 * NLEG + 1][lane], lds.cap[2 * NLEG + 2][lane],
                             lds.cap[2 * NLEG + 3][lane]};
      const float w[3] = {lds.cap[2 * NLEG + 4][lane], lds.cap[2 * NLEG + 5][lane], lds.cap[2 * NLEG + 6][lane]};
      capture_imu(quat, w, imu_dst);
    }
#pragma unroll
    for (int k = 0; k < NLEG; ++k) {
      B.dof_state[n * 24 + 2 * (j0 + k)] = q[k];
      B.dof_state[n * 24 + 2 * (j0 + k) + 1] = qd[k];
      B.torques[n * 12 + j0 + k] = tau[k];
    }
  }
  float (*FR)[NE5] = FUSED ? lds.fr : nullptr;
  if constexpr (FUSED) {
#pragma unroll
    for (int k = 0; k < NLEG; ++k) {
      lds.fr[F_DOF + 2 * (j0 + k)][e] = q[k];
      lds.fr[F_DOF + 2 * (j0 + k) + 1][e] = qd[k];
      lds.fr[F_TQ + j0 + k][e] = tau[k];
    }
  }
  __syncthreads();  // R1: the end-of-step state published (W3 computes the contact forces meanwhile)
  T1_PROF_MARK(9);
  {
    BaseFrame<float> F;
    base_frame(sb, F);
    leg_report_rigid<NE5>(M, B, PB, sb, F, q, qd, n, leg, active, e, FR);
  }
  T1_PROF_MARK(10);
  __syncthreads();  // RB: the contact-force report's parts in LDS (W1-W3 store it)
  if constexpr (FUSED) {
    __syncthreads();  // the epilogue barrier: every output of the workgroup is in LDS / memory
    T1_PROF_MARK(11);
    fused_epilogue_staged<POST_A_REWARDS, NE5, SH>(M, C, B, A, S, FA, dyn_blocks, lane, lds.epi, lds.fr, lds.act,
                                                     lds.act + NLEG);
  }
  T1_PROF_END();
}

#ifdef T1_PHASE_PROF
// profiling build only: summed clock deltas per [wave][bucket] since the last reset
extern "C" int t1env_debug_phase_cycles5(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_t1_prof5), sizeof(g_t1_prof5));
  if (e == hipSuccess && reset) {
    static const unsigned long long zero[T1_PROF_WAVES5][T1_NPROF5] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_t1_prof5), zero, sizeof(zero));
  }
  return (int)e;
}
#endif

int t1_launch_dyn5(const DynModel* d_model, const t1env_config* d_cfg, const t1env_buffers& B, const Terrain& T,
                   const float* actions, const t1env_step_args& A, int num_envs, const ShiftArgs& S,
                   const FusedArgs* fused, hipStream_t s, const SubLog* log, bool inwg_shift) {
  const int blocks = (num_envs + NE5 - 1) / NE5;
  const FusedArgs FA = fused ? *fused : FusedArgs{};
  const SubLog LG = log ? *log : SubLog{};
  const bool hf = T.type != 0;
  if (log && !fused) return (int)hipErrorInvalidValue;  // the substep log: fused steps only (the caller checks)
#define T1_LAUNCH5(HF, FU, SH) \
  hipLaunchKernelGGL((k_dyn5<HF, FU, SH>), dim3(blocks), dim3(D5_BLOCK), 0, s, d_model, d_cfg, B, T, actions, A, S, blocks, FA, LG)
  if (inwg_shift) {
    if (fused) { if (hf) T1_LAUNCH5(true, true, true); else T1_LAUNCH5(false, true, true); }
    else { if (hf) T1_LAUNCH5(true, false, true); else T1_LAUNCH5(false, false, true); }
  } else {
    if (fused) { if (hf) T1_LAUNCH5(true, true, false); else T1_LAUNCH5(false, true, false); }
    else { if (hf) T1_LAUNCH5(true, false, false); else T1_LAUNCH5(false, false, false); }
  }
#undef T1_LAUNCH5
  return (int)hipGetLastError();
}

