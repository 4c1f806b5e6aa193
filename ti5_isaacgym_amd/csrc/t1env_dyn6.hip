// t1env_dyn6.hip -- k_dyn6, the env step's main launch on eight waves: two waves per SIMD at 8192 envs
// (legged_robot.py:399-434 + Isaac Gym simulate(), and in the fused step post-physics, legged_robot.py:458-506).
//
// k_dyn5 (t1env_dyn5.hip) runs 32 envs per workgroup on four role waves, one wave per SIMD: every role is issue-bound at
// the lone-wave rate (one VALU instruction per 4 cycles, MI355X_MICROARCH.md constants table), and the step is the
// longest pre-S2 role (the shank + foot-half terrain wave, ~3.4k VALU instructions per substep) plus the core wave's
// post-S2 chain (~1.5k).  A SIMD issues a wave64 instruction in 2 cycles, so two waves per SIMD can double its VALU
// rate; k_dyn6 keeps k_dyn5's lane layout (lane l of a wave: env blockIdx.x * 32 + (l & 31), leg l >> 5) and its
// arithmetic, and spreads the pre-S2 work of the substep over eight roles of ~1.3-2k instructions, two per SIMD
// (waves w and w + 4 share SIMD w):
//
//   wave  SIMD  S1 -> S2 (the terms of the published state)            S2 -> S1
//   W0    0     pose chain + contact-free CRBA backward pass             core chain: fold-in, elimination, base system,
//                                                                        solve, back-substitution, integration, publish
//   W4    0     PD torques, base block, base-box contacts (both halves)  --
//   W1    1     RNEA bias and joint rhs                                  history shift slice
//   W5    1     self-contacts (capsules, both legs' bodies by permlane)  history shift slice
//   W2    2     shank terrain contact, points 0-3                        history shift slice
//   W6    2     shank terrain contact, points 4-7 (at S1: the sensor-lag  history shift slice
//               capture and substep log of the previous substep's state)
//   W3    3     foot terrain contact, points 0-3                         history shift slice
//   W7    3     foot terrain contact, points 4-7                         history shift slice
//
// The core wave (W0) owns the restitution episodes of the shank and foot: the contact halves publish the fastest
// approach of their points (amx), and W0 folds the two halves of a body into its episode after S2 (W4 keeps the base
// box's, as k_dyn5's W1).  The history shift is not staged in LDS (the role hand-offs need it): each of the six shift
// waves copies one tenth of its share of the workgroup's rows per substep through VGPRs, pipelined across the substep
// -- slice s + 1's two aligned 16-B source loads per output chunk are issued right after slice s's stores and held in
// registers through the next substep's role work (ShiftHold), so the HBM stream spans the whole substep -- and stores
// whole 16-B chunks (the newest frame of a row is a don't-care the epilogue rewrites; only the workgroup's last chunk
// takes an element path).  The step's report and the fused epilogue are k_dyn5's, spread over the eight waves.
//
// Every value is computed by the same t1_dynamics.h / t1_dyn5.h functions as in k_dyn5; what differs is the order of a
// few sums: a contact body's terms are the sum of its two point halves (and the self terms) instead of one 8-point
// accumulation.  compute_delta_roles6 (t1_dyn5.h) is the same composition on one host thread (tests/test_dynamics.py).
#include <hip/hip_runtime.h>

// one inlined copy of the contact law per call site (body_contact_fixed_q, contact_half) instead of a copy
// specialised for waves without a restitution set point: the -O2 build merged the two and indexed a scratch copy of
// the query (-DT1_D6_VTG_SPECIALIZE: the two copies, A/B)
#ifndef T1_D6_VTG_SPECIALIZE
#define T1_CONTACT_ONE_COPY
#endif

#ifdef T1_PROBE_SIMD
// probe build only: the hardware placement of every wave of the last launch (HW_ID: SIMD, CU, SE), [block][wave]
__device__ unsigned g_t1_simd6[4096][8];
#endif
#ifdef T1_PROBE_CLOCK
// probe build only (tools/clock_probe.py): per workgroup, W0's shader cycles (s_memtime) and 100 MHz constant-clock
// ticks (s_memrealtime) from its start to the end of its epilogue, summed over workgroups and launches, and the count
__device__ unsigned long long g_t1_clock6[4];
// and the timeline of the last launch, per workgroup: {start, W0 end, last wave's end} in 100 MHz ticks; per workgroup
// summed over launches: {W0 lifetime, W0's S1 waits, W0's S2 waits} in shader cycles
__device__ unsigned long long g_t1_wgtime6[4096][4];  // + [3]: W0's substep loop end
__device__ unsigned long long g_t1_wgsum6[4096][3];
#define T1_CLOCK_WAIT_BEGIN() const unsigned long long t1c_w0 = __builtin_amdgcn_s_memtime();
#define T1_CLOCK_LOOP_END()                                                        \
  if (threadIdx.x == 0 && blockIdx.x < 4096) g_t1_wgtime6[blockIdx.x][3] = __builtin_amdgcn_s_memrealtime();
#define T1_CLOCK_WAIT_END(k)                                                       \
  if (threadIdx.x == 0 && blockIdx.x < 4096)                                       \
    atomicAdd(&g_t1_wgsum6[blockIdx.x][k], __builtin_amdgcn_s_memtime() - t1c_w0);
#define T1_CLOCK_BEGIN()                                                           \
  unsigned long long t1c_cyc0 = 0, t1c_rt0 = 0;                                    \
  if (threadIdx.x == 0) {                                                          \
    t1c_cyc0 = __builtin_amdgcn_s_memtime();                                       \
    t1c_rt0 = __builtin_amdgcn_s_memrealtime();                                    \
    if (blockIdx.x < 4096) { g_t1_wgtime6[blockIdx.x][0] = t1c_rt0; g_t1_wgtime6[blockIdx.x][2] = 0; } \
  }
#define T1_CLOCK_END()                                                             \
  if (threadIdx.x == 0) {                                                          \
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime(); \
    atomicAdd(&g_t1_clock6[0], c1 - t1c_cyc0);                                     \
    atomicAdd(&g_t1_clock6[1], r1 - t1c_rt0);                                      \
    atomicAdd(&g_t1_clock6[2], 1ull);                                              \
    if (blockIdx.x < 4096) {                                                       \
      g_t1_wgtime6[blockIdx.x][1] = r1;                                            \
      atomicAdd(&g_t1_wgsum6[blockIdx.x][0], c1 - t1c_cyc0);                       \
    }                                                                              \
  }                                                                                \
  T1_CLOCK_WAVE_END();
#define T1_CLOCK_WAVE_END()                                                        \
  if ((threadIdx.x & 63) == 0 && blockIdx.x < 4096)                                \
    atomicMax(&g_t1_wgtime6[blockIdx.x][2], (unsigned long long)__builtin_amdgcn_s_memrealtime());
#else
#define T1_CLOCK_BEGIN() ((void)0)
#define T1_CLOCK_END() ((void)0)
#define T1_CLOCK_WAVE_END() ((void)0)
#define T1_CLOCK_WAIT_BEGIN() ((void)0)
#define T1_CLOCK_WAIT_END(k) ((void)0)
#define T1_CLOCK_LOOP_END() ((void)0)
#endif
// -DT1_PHASE_PROF (tools/prof_dynamics_phases.py --kernel 6): lane 0 of every wave accumulates shader-clock deltas
// between T1_PROF_MARK points into per-phase buckets; never part of the product build.
#ifdef T1_PHASE_PROF
constexpr int T1_NPROF6 = 24, T1_PROF_WAVES6 = 8;
__device__ unsigned long long g_t1_prof6[T1_PROF_WAVES6][T1_NPROF6];
__shared__ unsigned long long t1_prof_acc6[T1_PROF_WAVES6][T1_NPROF6 + 1];  // [wave][bucket], last = previous mark
__device__ __forceinline__ unsigned long long t1_stamp6() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
__device__ __forceinline__ void t1_prof_mark6(int i) {
  const int w = threadIdx.x / 64;
  const unsigned long long now = t1_stamp6();
  if ((threadIdx.x & 63) == 0) {
    t1_prof_acc6[w][i] += now - t1_prof_acc6[w][T1_NPROF6];
    t1_prof_acc6[w][T1_NPROF6] = now;
  }
}
__device__ __forceinline__ void t1_prof_begin6() {
  const int w = threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0) {
    for (int i = 0; i < T1_NPROF6; ++i) t1_prof_acc6[w][i] = 0;
    t1_prof_acc6[w][T1_NPROF6] = t1_stamp6();
  }
}
__device__ __forceinline__ void t1_prof_end6() {
  const int w = threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0)
    for (int i = 0; i < T1_NPROF6; ++i) atomicAdd(&g_t1_prof6[w][i], t1_prof_acc6[w][i]);
}
#define T1_PROF_MARK(i) t1_prof_mark6(i)
#define T1_PROF_BEGIN() t1_prof_begin6()
#define T1_PROF_END() t1_prof_end6()
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

constexpr int NE6 = 32;        // envs per workgroup
constexpr int D6_BLOCK = 512;  // eight waves

// W4 -> W0: the substep's PD torques, the base block with both base-box halves, its rhs
enum : int { WB_TAU = 0, WB_AC = 8, WB_R = 29, WB_N = 35 };
// W0's joint subspaces (its CRBA pass -> its fold-in), in rows of their own
struct SubspaceRows { float4 r[NLEG][2][64]; };  // S_k = (r[k][0], r[k][1].xy)
// W1 -> W0: the bias part of each joint rhs (-S_k . sum_{j>=k} g_j) and the leg's total bias
enum : int { R_RG = 0, R_G = 6, R_N = 12 };
// contact terms -> W0
enum : int { WC_SHA = 0, WC_SHB = 1, WC_FTA = 2, WC_FTB = 3, WC_SSH = 4, WC_SFT = 5, WC_N = 6 };
// the shift waves (post-S2) and their count
#ifndef T1_D6_SHIFT_MASK  // A/B builds: -DT1_D6_SHIFT_MASK=...
#define T1_D6_SHIFT_MASK ((1 << 1) | (1 << 5) | (1 << 2) | (1 << 6) | (1 << 3) | (1 << 7))
#endif
constexpr int SHIFT6_MASK = T1_D6_SHIFT_MASK;  // by role (below)
// the shift roles that commit their slice (and issue the next one's loads) before S2, in the slack their role work
// leaves ahead of the core wave's pre-S2 chain, instead of after S2 where the core wave may wait for them at S1
// (-DT1_D6_SHIFT_PRE_MASK=..., by role; 0: every shift role after S2)
#ifndef T1_D6_SHIFT_PRE_MASK
#define T1_D6_SHIFT_PRE_MASK 0
#endif
constexpr int SHIFT6_PRE_MASK = T1_D6_SHIFT_PRE_MASK;
// The role of each wave: role ids are the wave numbers of the table at the top (0 core, 4 base, 1 RNEA, 5 self, 2 / 6
// shank halves, 3 / 7 foot halves); T1_D6_ROLE_MAP holds the role of wave w in hex digit w, so the SIMD pairs (w, w + 4)
// can be re-dealt for A/B (the core stays wave 0: its partner is wave 4's role)
#ifndef T1_D6_ROLE_MAP
#define T1_D6_ROLE_MAP 0x76543210u
#endif
__device__ __forceinline__ int role_of(int wave) {
#ifdef T1_PROBE_ROLE  // register-probe builds only (every wave one role: the others' code compiled out)
  return T1_PROBE_ROLE;
#endif
  return (int)((T1_D6_ROLE_MAP >> (4 * wave)) & 0xFu);
}
static_assert((T1_D6_ROLE_MAP & 0xFu) == 0, "the core role is wave 0");
constexpr int SHIFT6_WAVES = __builtin_popcount(SHIFT6_MASK);
static_assert((SHIFT6_MASK & 0x11) == 0, "W0 / W4 (the core chain's SIMD) do not shift");

struct Dyn6Lds {
  DynModel model;
  Rows4<Q_N> st;          // W0 -> all: substep state
  Rows4<WB_N> wb;         // W4 -> W0
  SubspaceRows sj;        // W0
  Rows4<R_N> w1;          // W1 -> W0
  Rows4<XCH> wc[WC_N];    // contact roles -> W0
  PdStage<64> pd;         // W4: PD constants and action ring of each lane's leg
  float cap[CAP5_N][64];  // W6: the sensor-lag samples captured in the loop
  float act[12][NE6];     // the clipped actions (epilogue)
  float epi[EPI_N][NE6];  // staged post-physics inputs (epilogue)
  float fr[FR_N][NE6];    // this step's outputs (epilogue)
  float vish[64];         // the shank's restitution episode (W0 updates it after S2; W2 / W6 read it)
  float vift[64];         // the foot's (W0; W3 / W7)
  float amx[4][64];       // the fastest approach among the points of the shank halves [0, 1] and foot halves [2, 3]
  int s1flag;             // T1_D6_S1_FLAG: the number of substep states W0 has published (S1 as a one-way signal)
  LegParams<float> pl[64];   // W0's per-lane leg parameters (CRBA) and base parameters (report, log): LDS, not
  BaseParams<float> pb[64];  // registers held across the substep loop
  float rtf[2][3][64];    // the report: terrain forces on the shank [0] (W2) / foot [1] (W3)
  float rsf[2][3][64];    // the report: self-contact forces on the shank / foot (W5)
};

// ---- the history shift through VGPRs.  Output element e of a row-major history (rows of ROW = F * H) is input element
// e + F unless e is in the row's newest frame (column >= ROW - F), which the epilogue (or k_post_b) of the same
// workgroup writes after the shift has completed.  So a 16-B output chunk is stored whole -- its newest-frame elements
// are don't-cares -- whenever it lies inside the workgroup's rows and its two aligned 16-B source blocks inside the
// buffer; only a chunk crossing into the next workgroup's first row (whose epilogue may zero it for a reset: the race
// the whole-chunk store must not enter) or sourcing past the buffer's end takes the element path.
// bytes [OFF, OFF + 16) of the 32-B window a:b
template <uint32_t OFF>
__device__ __forceinline__ u32x4 shift_window(const float4& a, const float4& b) {
  const u32x4 xa = __builtin_bit_cast(u32x4, a), xb = __builtin_bit_cast(u32x4, b);
  const uint32_t w[8] = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w};
  constexpr uint32_t M = OFF / 4, R = OFF % 4;
  if constexpr (R == 0) {
    return u32x4{w[M], w[M + 1], w[M + 2], w[M + 3]};
  } else {
    return u32x4{__builtin_amdgcn_alignbyte(w[M + 1], w[M], R), __builtin_amdgcn_alignbyte(w[M + 2], w[M + 1], R),
                 __builtin_amdgcn_alignbyte(w[M + 3], w[M + 2], R), __builtin_amdgcn_alignbyte(w[M + 4], w[M + 3], R)};
  }
}
// the element path of one chunk (elements [i, i + PER) of the workgroup's nel): older-frame columns only
template <int F, int H, bool HALF>
__device__ __forceinline__ void shift_chunk_elems(const uint8_t* in0, uint8_t* out0, uint32_t i, uint32_t nel) {
  constexpr uint32_t ROW = F * H, PER = HALF ? 8 : 4;
#pragma unroll 1
  for (uint32_t k = 0; k < PER; ++k) {
    const uint32_t e = i + k;
    if (e < nel && e % ROW < ROW - F) {
      if constexpr (HALF)
        reinterpret_cast<uint16_t*>(out0)[e] = reinterpret_cast<const uint16_t*>(in0)[e + F];
      else
        reinterpret_cast<float*>(out0)[e] = reinterpret_cast<const float*>(in0)[e + F];
    }
  }
}
// the chunk range [lo, hi) of slice sl of one history of the rows [r0, r1); lim: elements to the buffer's end, nel:
// the workgroup's elements (its rows, clipped to the buffer)
template <int F, int H, bool HALF>
__device__ __forceinline__ void shp_range(int64_t total, int64_t r0, int64_t r1, int sl, int nsl, uint32_t& lo,
                                          uint32_t& hi, uint32_t& lim, uint32_t& nel) {
  constexpr uint32_t ROW = F * H, PER = HALF ? 8 : 4;
  lim = (uint32_t)(total - r0 * (int64_t)ROW);
  const uint32_t span = (uint32_t)((r1 - r0) * ROW);
  nel = span < lim ? span : lim;
  const uint32_t n = (nel + PER - 1) / PER;
  lo = n * (uint32_t)sl / (uint32_t)nsl;
  hi = n * (uint32_t)(sl + 1) / (uint32_t)nsl;
}
// One 16-B load from the exact source of a chunk (4-byte aligned for fp32 histories, 2-byte for fp16) -- the hardware
// serves an unaligned dwordx4 (the unaligned access mode ROCm sets for gfx9; tools/probes/unaligned_x4.hip) -- instead
// of the two aligned blocks around it and an alignbyte window (-DT1_D6_SHIFT_ALIGNED2, A/B): half the load instructions
// of a slice and half the registers held across the substep (ShiftHold::b unused)
#ifndef T1_D6_SHIFT_ALIGNED2
constexpr bool SHIFT_EXACT32 = true;
#else
constexpr bool SHIFT_EXACT32 = false;
#endif
typedef float shift_f4 __attribute__((ext_vector_type(4)));
// the source loads of U chunks (lane t0's, `stride` apart from chunk lo)
template <int F, bool HALF, int U>
__device__ __forceinline__ void shift_loads(const uint8_t* in0, uint32_t lo, uint32_t lim, int t0, int stride,
                                            float4* a, float4* b) {
  constexpr uint32_t PER = HALF ? 8 : 4, ES = HALF ? 2 : 4;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t c = lo + (uint32_t)(t0 + u * stride);
    if constexpr (SHIFT_EXACT32) {
      const uint32_t src = c * PER + F;
      const uint32_t sc = src + PER <= lim ? src : lim - PER;  // tail: an in-bounds dummy
      const shift_f4 v = *reinterpret_cast<const shift_f4*>(in0 + (size_t)sc * ES);
      a[u] = make_float4(v.x, v.y, v.z, v.w);
    } else {
      const uint32_t sa = (c * PER + F) & ~(PER - 1);
      const uint32_t sc = sa + 2 * PER <= lim ? sa : (lim - 2 * PER) & ~(PER - 1);  // tail: an aligned in-bounds dummy
      a[u] = *reinterpret_cast<const float4*>(in0 + (size_t)sc * ES);
      b[u] = *reinterpret_cast<const float4*>(in0 + (size_t)(sc + PER) * ES);
    }
  }
}
// the stores of U chunks from their loaded source blocks (whole chunks; the rest by the element path)
template <int F, int H, bool HALF, int U>
__device__ __forceinline__ void shift_stores(const uint8_t* in0, uint8_t* out0, uint32_t lo, uint32_t hi,
                                             uint32_t lim, uint32_t nel, int t0, int stride, const float4* a,
                                             const float4* b) {
  constexpr uint32_t PER = HALF ? 8 : 4, ES = HALF ? 2 : 4, OFF = (F * ES) % 16;
  uint32_t slow = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t c = lo + (uint32_t)(t0 + u * stride), i = c * PER;
    if constexpr (SHIFT_EXACT32) {
      if (c < hi) {
        if (i + PER <= nel && i + F + PER <= lim)
          __builtin_nontemporal_store(__builtin_bit_cast(u32x4, a[u]), reinterpret_cast<u32x4*>(out0 + (size_t)i * ES));
        else
          slow |= 1u << u;
      }
    } else {
      const uint32_t sa = (i + F) & ~(PER - 1);
      if (c < hi) {
        if (i + PER <= nel && sa + 2 * PER <= lim)
          __builtin_nontemporal_store(shift_window<OFF>(a[u], b[u]), reinterpret_cast<u32x4*>(out0 + (size_t)i * ES));
        else
          slow |= 1u << u;
      }
    }
  }
  if (slow) {
#pragma unroll 1
    for (int u = 0; u < U; ++u)
      if ((slow >> u) & 1u) shift_chunk_elems<F, H, HALF>(in0, out0, (lo + (uint32_t)(t0 + u * stride)) * PER, nel);
  }
}
// chunks [c_lo, c_hi) of the workgroup's rows, U per lane per round, every round's loads before its stores
template <int F, int H, bool HALF, int U>
__device__ __forceinline__ void shift6_range(const uint8_t* in0, uint8_t* out0, uint32_t c_lo, uint32_t c_hi,
                                             uint32_t lim, uint32_t nel, int t0, int stride) {
  for (uint32_t base = c_lo; base + (uint32_t)t0 < c_hi; base += U * (uint32_t)stride) {
    float4 a[U], b[U];
    shift_loads<F, HALF, U>(in0, base, lim, t0, stride, a, b);
    shift_stores<F, H, HALF, U>(in0, out0, base, c_hi, lim, nel, t0, stride, a, b);
  }
}
// ---- the shift pipelined across the substep: a shift wave issues the source loads of slice s + 1 right after it
// stores slice s (after S2), holds them in registers through substep s + 1's role work (the HBM stream then spans the
// whole substep instead of the post-S2 window alone, where its burst outlasted the core chain) and forms and stores
// the outputs after the next S2.  A lane holds U_O chunks of the actor history and one of the critic history; a slice
// with more chunks (fewer than 10 substeps) does the rest through shift6_f32 / _f16 at commit time.
constexpr int SHP_UO = 7, SHP_UP = 1;  // 32 rows / 10 slices / (6 x 64) lanes: 6.5 actor chunks, 0.5 critic
struct ShiftHold {
  float4 a[SHP_UO + SHP_UP], b[SHP_UO + SHP_UP];  // the two aligned 16-B source blocks of each held chunk
};
template <int F, int H, bool HALF, int U>
__device__ __forceinline__ void shp_issue(const void* in, int64_t total, int64_t r0, int64_t r1, int sl, int nsl,
                                          int t0, int stride, float4* a, float4* b) {
  constexpr uint32_t ROW = F * H, ES = HALF ? 2 : 4;
  uint32_t lo, hi, lim, nel;
  shp_range<F, H, HALF>(total, r0, r1, sl, nsl, lo, hi, lim, nel);
  shift_loads<F, HALF, U>(reinterpret_cast<const uint8_t*>(in) + (size_t)(r0 * ROW) * ES, lo, lim, t0, stride, a, b);
}
template <int F, int H, bool HALF, int U>
__device__ __forceinline__ void shp_commit(const void* in, void* out, int64_t total, int64_t r0, int64_t r1, int sl,
                                           int nsl, int t0, int stride, const float4* a, const float4* b) {
  constexpr uint32_t ROW = F * H, ES = HALF ? 2 : 4;
  uint32_t lo, hi, lim, nel;
  shp_range<F, H, HALF>(total, r0, r1, sl, nsl, lo, hi, lim, nel);
  const uint8_t* in0 = reinterpret_cast<const uint8_t*>(in) + (size_t)(r0 * ROW) * ES;
  uint8_t* out0 = reinterpret_cast<uint8_t*>(out) + (size_t)(r0 * ROW) * ES;
  shift_stores<F, H, HALF, U>(in0, out0, lo, hi, lim, nel, t0, stride, a, b);
  // chunks past the held ones (a slice larger than the lanes hold: fewer than 10 substeps)
  const uint32_t rest = lo + (uint32_t)(U * stride);
  if (rest < hi) shift6_range<F, H, HALF, 1>(in0, out0, rest, hi, lim, nel, t0, stride);
}
// issue slice sl's loads into H (shift wave wi); commit slice sl from H
__device__ __forceinline__ void shp_issue_slice(const ShiftArgs& S, int64_t r0, int64_t r1, int sl, int nsl, int wi,
                                                int lane, ShiftHold& Hd) {
#ifdef T1_WHATIF_D6_NO_SHIFT
  return;
#endif
  if (r1 <= r0 || sl >= nsl) return;
  const int t0 = wi * 64 + lane, stride = 64 * SHIFT6_WAVES;
  if (S.half) {
    shp_issue<T1_NOBS, T1_HIST, true, SHP_UO>(S.obs_in, S.total_obs, r0, r1, sl, nsl, t0, stride, Hd.a, Hd.b);
    shp_issue<T1_NPRIV, T1_CHIST, true, SHP_UP>(S.priv_in, S.total_priv, r0, r1, sl, nsl, t0, stride, Hd.a + SHP_UO,
                                                Hd.b + SHP_UO);
  } else {
    shp_issue<T1_NOBS, T1_HIST, false, SHP_UO>(S.obs_in, S.total_obs, r0, r1, sl, nsl, t0, stride, Hd.a, Hd.b);
    shp_issue<T1_NPRIV, T1_CHIST, false, SHP_UP>(S.priv_in, S.total_priv, r0, r1, sl, nsl, t0, stride, Hd.a + SHP_UO,
                                                 Hd.b + SHP_UO);
  }
}
__device__ __forceinline__ void shp_commit_slice(const ShiftArgs& S, int64_t r0, int64_t r1, int sl, int nsl, int wi,
                                                 int lane, const ShiftHold& Hd) {
#ifdef T1_WHATIF_D6_NO_SHIFT
  return;
#endif
  if (r1 <= r0 || sl >= nsl) return;
  const int t0 = wi * 64 + lane, stride = 64 * SHIFT6_WAVES;
  const ShiftHold& H = Hd;
  if (S.half) {
    shp_commit<T1_NOBS, T1_HIST, true, SHP_UO>(S.obs_in, S.obs_out, S.total_obs, r0, r1, sl, nsl, t0, stride, H.a,
                                               H.b);
    shp_commit<T1_NPRIV, T1_CHIST, true, SHP_UP>(S.priv_in, S.priv_out, S.total_priv, r0, r1, sl, nsl, t0, stride,
                                                 H.a + SHP_UO, H.b + SHP_UO);
  } else {
    shp_commit<T1_NOBS, T1_HIST, false, SHP_UO>(S.obs_in, S.obs_out, S.total_obs, r0, r1, sl, nsl, t0, stride, H.a,
                                                H.b);
    shp_commit<T1_NPRIV, T1_CHIST, false, SHP_UP>(S.priv_in, S.priv_out, S.total_priv, r0, r1, sl, nsl, t0, stride,
                                                  H.a + SHP_UO, H.b + SHP_UO);
  }
}

__device__ __forceinline__ int shift6_index(int role) {  // the role's index among the shifting roles, -1: none
  return (SHIFT6_MASK >> role) & 1 ? __builtin_popcount(SHIFT6_MASK & ((1 << role) - 1)) : -1;
}

// The model in LDS as the loop sees it: the address passes through an empty asm each substep, so its per-lane reads (the
// leg index is a lane value) are not hoisted out of the substep loop as invariants -- at two waves per SIMD (256
// registers) the hoisted model values would be spilled to scratch, and an LDS read is the cheaper re-load
__device__ __forceinline__ const DynModel& model_in_loop(const DynModel& m) {
  typedef __attribute__((address_space(3))) const DynModel* lds_model_ptr;
  lds_model_ptr p = (lds_model_ptr)&m;
  asm volatile("" : "+s"(p));
  return *(const DynModel*)p;
}

// S1 as a one-way signal (-DT1_D6_S1_FLAG): W0 publishes the substep state and counts it in an LDS word instead of
// meeting the other seven waves at a workgroup barrier, so it starts its next pre-S2 chain at once; a role wave waits
// for the count before it reads the state.  What S1 also ordered still holds: W0 finishes its reads of the role rows
// (wb, w1, wc, amx) before it publishes, and the role waves write them only after the count, and S2 (a full barrier)
// keeps W0 from publishing over a state a role still reads.  The wait is bounded (it never runs long: W0 signals
// every substep), so a fault cannot turn into a hang.
__device__ __forceinline__ void s1_signal(int* flag, int value) {
  __hip_atomic_store(flag, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void s1_wait(int* flag, int target) {
  for (int i = 0; i < (1 << 22); ++i) {
    const int v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
    if (v >= target) break;
    __builtin_amdgcn_s_sleep(1);
  }
}
#ifdef T1_D6_S1_FLAG
#define D6_S1(target) s1_wait(&lds.s1flag, (target))
#else
#define D6_S1(target) __syncthreads()
#endif

// the other leg's capsule ends and velocity (from the other half of the wave) for the self-contact terms / forces
__device__ __forceinline__ void self_bodies(const DynModel& M, int leg, const BodyKin<float> (&Ko)[2],
                                            SelfBody<float> (&O)[2], SelfBody<float> (&X)[2]) {
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
}

// one contact half (4 points) of the shank or foot against the terrain: its terms and the fastest approach of its
// points (amax < 0: none in contact, or the body out of the terrain's reach by its height bound -- the shank only)
template <bool HF, bool BOUND>
__device__ __forceinline__ void contact_half(const DynModel& M, const Terrain& T, int c0, const BodyKin<float>& K,
                                             const BaseFrame<float>& F, int b, float mu, float vtg, float dt,
                                             Sym6<float>& C, float c[6], float& amax) {
  ContactQuery<T1_POINTS_PER_BODY / 2, float> Q;
  contact_query<HF, T1_POINTS_PER_BODY / 2>(M, T, c0, K.Rb, K.p, F.abs, Q);
  amax = -1.0f;
  if constexpr (BOUND) {  // the body's height bound, loaded with the point queries (one memory round trip)
    const int32_t bnd = terrain_bound_raw_any(T, K.p.x + F.abs.x, K.p.y + F.abs.y);
    if (K.p.z + F.abs.z - M.contact_radius[b] > bound_height<float>(T, bnd)) return;
  }
#ifdef T1_D6_VTG_SPECIALIZE  // A/B: the contact law specialised for a wave without a restitution set point
  if (t1_wave_any(vtg > 0.0f)) contact_apply<HF, T1_POINTS_PER_BODY / 2>(M, Q, K.V, mu, vtg, dt, C, c, amax);
  else contact_apply<HF, T1_POINTS_PER_BODY / 2>(M, Q, K.V, mu, 0.0f, dt, C, c, amax);
#else  // one copy of the contact law (the -O2 build merged the two and indexed a scratch copy of Q)
  contact_apply<HF, T1_POINTS_PER_BODY / 2>(M, Q, K.V, mu, vtg, dt, C, c, amax);
#endif
}

// leg_apply_terms (t1_dyn5.h) with its inputs read from LDS where they are used, to hold the core wave's register peak:
// the joint subspaces (W0's own CRBA rows) per joint, the foot's terms ((points 0-3 + 4-7) + self) for joints 5 and 4,
// then the shank's, added to them in place for joints 3-0 (Cs = C0 + C1, the same sums), the bias G last.  Every
// element gets leg_apply_terms' operations in its order (the L, Bl and rhs updates of different joints are independent).
template <int K0, int K1>
__device__ __forceinline__ void leg_apply_terms_rows(const Rows4<XCH> (&W)[WC_N], const Rows4<R_N>& W1,
                                                     const float rg[NLEG], const SubspaceRows& SR, int lane,
                                                     LegBlock<float>& out, Sym6<float>& Ac_up, float gc_up[6]) {
  static_assert(K0 == K_SHANK && K1 == K_FOOT && K1 == NLEG - 1, "the foot's terms first, then the shank's");
  auto terms = [&](int i, Sym6<float>& Cb, float cb[6]) {  // contact body i (0 shank, 1 foot): (half 0 + half 1) + self
    float va[XCH];
    get4(W[2 * i], lane, va);
    {
      float vb[XCH];
      get4(W[2 * i + 1], lane, vb);
#pragma unroll
      for (int k = 0; k < XCH; ++k) va[k] = va[k] + vb[k];
    }
    {
      float vs[XCH];
      get4(W[WC_SSH + i], lane, vs);
#pragma unroll
      for (int k = 0; k < XCH; ++k) va[k] = va[k] + vs[k];
    }
    sym_unpack(va, Cb, cb);
  };
  auto subspace = [&](int k, float (&Sk)[6]) {
    const float4 x = SR.r[k][0][lane], y = SR.r[k][1][lane];
    Sk[0] = x.x; Sk[1] = x.y; Sk[2] = x.z; Sk[3] = x.w; Sk[4] = y.x; Sk[5] = y.y;
  };
  Sym6<float> C;  // C1 (the foot), then Cs = C0 + C1
  float c[6];
  terms(1, C, c);
  auto joint = [&](auto jc) {
    constexpr int jj = decltype(jc)::value;
    float Sj[6], u[6];
    subspace(jj, Sj);
    sym_mul(C, Sj, u);
    const float sc = dot6(Sj, c);
    out.L[sidx(jj, jj)] += dot6(Sj, u);
    out.rhs[jj] += rg[jj] - sc;
#pragma unroll
    for (int k = 0; k < jj; ++k) {
      float Sk[6];
      subspace(k, Sk);
      out.L[sidx(k, jj)] += dot6(Sk, u);
    }
#pragma unroll
    for (int r = 0; r < 6; ++r) out.Bl[r][jj] += u[r];
  };
  joint(kconst<5>{});
  joint(kconst<4>{});
  {
    Sym6<float> C0;
    float c0[6];
    terms(0, C0, c0);
#pragma unroll
    for (int i = 0; i < 21; ++i) C.a[i] = C0.a[i] + C.a[i];
#pragma unroll
    for (int i = 0; i < 6; ++i) c[i] = c0[i] + c[i];
  }
  joint(kconst<3>{});
  joint(kconst<2>{});
  joint(kconst<1>{});
  joint(kconst<0>{});
  sym_add(Ac_up, C);
  float w1v[R_N];
  get4(W1, lane, w1v);
#pragma unroll
  for (int i = 0; i < 6; ++i) gc_up[i] += w1v[R_G + i] + c[i];
}

// The state after substep s, recorded by W6 (it reads that state at the next S1, the last one after R1): the sensor-lag
// samples the next observation reads (the joint state at substep 9 - lag % 10, the raw IMU sample likewise) into LDS,
// and the substep log's rows (tests only; LG.root is a wave-uniform kernel argument)
__device__ __forceinline__ void record_substep(const DynModel& M, const BaseParams<float>& PB, const SubLog& LG,
                                               Dyn6Lds& L, int s, int s_dof, int s_imu, int N, int n, int j0, int leg,
                                               int lane, bool active, const BaseState<float>& sb,
                                               const float (&q)[NLEG], const float (&qd)[NLEG]) {
  if (LG.root != nullptr && active) {
    const size_t row = (size_t)s * N + n;
#pragma unroll
    for (int k = 0; k < NLEG; ++k) {
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
  if (s == s_dof) {
#pragma unroll
    for (int k = 0; k < NLEG; ++k) { L.cap[k][lane] = q[k]; L.cap[NLEG + k][lane] = qd[k]; }
  }
  if (leg == 0 && s == s_imu) {
#pragma unroll
    for (int i = 0; i < 4; ++i) L.cap[2 * NLEG + i][lane] = sb.quat[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) L.cap[2 * NLEG + 4 + i][lane] = sb.w[i];
  }
}

template <bool HF, bool FUSED>
__global__ __launch_bounds__(D6_BLOCK) void k_dyn6(const DynModel* __restrict__ Mg, const t1env_config* __restrict__ Cp,
                                                   t1env_buffers B, Terrain Tin, const float* __restrict__ actions,
                                                   t1env_step_args A, ShiftArgs S, int dyn_blocks, FusedArgs FA,
                                                   SubLog LG) {
  __shared__ Dyn6Lds lds;
  T1_CLOCK_BEGIN();
  {  // the model to LDS
    constexpr int NW = (int)(sizeof(DynModel) / 4);
    static_assert(sizeof(DynModel) % 4 == 0, "the model copies as words");
    const uint32_t* src = reinterpret_cast<const uint32_t*>(Mg);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&lds.model);
    for (int i = threadIdx.x; i < NW; i += D6_BLOCK) dst[i] = src[i];
  }
  Terrain T = Tin;
  T.type = HF ? 2 : 0;
  const t1env_config& C = *Cp;
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x / 64);
  const int role = role_of(wave);
#ifdef T1_PROBE_SIMD
  if ((threadIdx.x & 63) == 0 && blockIdx.x < 4096) g_t1_simd6[blockIdx.x][wave] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
#endif
  const int lane = threadIdx.x & 63;
  const int leg = lane >> 5;
  const int e = lane & 31;
  const int j0 = 6 * leg;
  const int N = C.num_envs;
  const int n0 = (int)blockIdx.x * NE6 + e;
  const bool active = n0 < N;
  const int n = active ? n0 : N - 1;
  const float dt = C.sim_dt;
  const uint32_t ctr = A.counter;
  const int nsub = C.decimation;
  const int64_t r0 = (int64_t)blockIdx.x * NE6, r1 = r0 + NE6 < N ? r0 + NE6 : N;
  T1_PROF_BEGIN();
  if (threadIdx.x == 0) lds.s1flag = 0;
  __syncthreads();  // the model in LDS
  const DynModel& M = lds.model;

  if (role == 4) {
    // ======== W4: base -- the actions, PD torques, the base block and both base-box halves (their restitution episode)
    const BaseParams<float>& PB = lds.pb[lane];  // W0 stores it before the first S1 (LDS, not registers held across
                                                 // the loop); read from the first substep on
    // the friction and restitution, lag, force and episode loads, then the actions and PD constants below, before the
    // first global store (the buffers may alias as far as the compiler knows)
#ifdef T1_D6_STAGE_FIRST  // A/B: the staging loads first (0.1275 vs 0.1270 ms, r05st: not kept)
    EpiStage<NE6, 256> EV;
    if (FUSED) epi_stage_load<NE6, 256>(B, N, (int)r0, (int)threadIdx.x - 256, EV);
#endif
#ifdef T1_PROBE_SCRATCH  // probe build only: a 64-B per-lane scratch object, touched once in W4's prologue
    {
      volatile float pad[16];
      pad[lane & 15] = 1.0f;
      if (pad[(lane + 3) & 15] == 12345.0f) B.torques[0] = 0.0f;
    }
#endif
    const float mu = 0.5f * (B.friction[n] + M.ground_friction);  // load_base_params' friction, restitution
    const float eg = ground_restitution(M, B.restitution[n]);
    const int lag = B.lag_timestep[n];
    const RngKey K = rng_key(C.seed, (uint32_t)(C.env_offset + n), ctr);
    const V3<float> ef = v3<float>(B.applied_force[n * 3 + 0], B.applied_force[n * 3 + 1], B.applied_force[n * 3 + 2]);
    float vi_b = B.contact_vimp[(size_t)n * NVIMP + vimp_base(leg)];
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
    // the epilogue's inputs the step does not change, staged by W4-W7 before their first substep (staged by W4 alone
    // in the first substep's idle S2 -> S1 window instead: 0.1301 vs 0.1269 ms, its loop's registers spill, r05stage)
#ifdef T1_D6_STAGE_FIRST
    if (FUSED) epi_stage_store<NE6, 256>(N, (int)r0, (int)threadIdx.x - 256, EV, lds.epi);
#else
    if (FUSED) stage_epilogue_inputs<NE6, 256>(B, N, (int)r0, (int)threadIdx.x - 256, lds.epi);
#endif
    int cb, ce;
    base_contact_range(M, leg, cb, ce);
    T1_PROF_MARK(0);
    for (int sub = 0; sub < nsub; ++sub) {
      D6_S1(sub + 1);  // S1: the substep state published
      T1_PROF_MARK(1);
      const DynModel& M = model_in_loop(lds.model);
      BaseState<float> sb;
      float q[NLEG], qd[NLEG];
      read_state_rows(lds.st, lane, sb, q, qd);
      BaseFrame<float> F;
      base_frame(sb, F);
      // the base box half's queries issued first, under the PD torques and the base block
      const int32_t bound_b = terrain_bound_raw_any(T, F.abs.x, F.abs.y);
      ContactQuery<T1_POINTS_PER_BODY / 2, float> Qb;
      contact_query<HF, T1_POINTS_PER_BODY / 2>(M, T, cb, F.R0, v3<float>(0, 0, 0), F.abs, Qb);
      float tau[NLEG];
      pd_torques_staged(M, C, lds.pd, lane, K, ctr, sub, lag, j0, q, qd, tau);
      Sym6<float> Ac;  // the base body's block (both halves compute it: the same values)
      float r[6];
      base_block(M, PB, F, sub == 0 ? ef : v3<float>(0, 0, 0), dt, Ac, r);
      {  // the base-box halves, summed left first (the same sum in both halves), into the base block
        Sym6<float> Cb;
        float gw[6] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
        sym_zero(Cb);
        body_contact_fixed_q<HF, T1_POINTS_PER_BODY / 2>(M, Qb, F.abs.z - M.contact_radius[0], bound_b, T, F.V0, mu, eg,
                                                         vi_b, dt, Cb, gw);
#pragma unroll
        for (int i = 0; i < 21; ++i) {
          float l, rr;
          halves(Cb.a[i], l, rr);
          Ac.a[i] = Ac.a[i] + (l + rr);
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          float l, rr;
          halves(gw[i], l, rr);
          r[i] = -r[i] + (-l - rr);
        }
      }
      float v[WB_N];
#pragma unroll
      for (int k = 0; k < NLEG; ++k) v[WB_TAU + k] = tau[k];
      v[NLEG] = 0.0f;
      v[NLEG + 1] = 0.0f;
#pragma unroll
      for (int i = 0; i < 21; ++i) v[WB_AC + i] = Ac.a[i];
#pragma unroll
      for (int i = 0; i < 6; ++i) v[WB_R + i] = r[i];
      put4(lds.wb, lane, v);
      if (LG.root != nullptr && active)  // the substep log's torques (tests only; wave-uniform kernel argument)
#pragma unroll
        for (int k = 0; k < NLEG; ++k) LG.torque[((size_t)sub * N + n) * 12 + j0 + k] = tau[k];
      T1_PROF_MARK(2);
      __syncthreads();  // S2: the terms published
      T1_PROF_MARK(3);
    }
    float tau[8];  // the last substep's torques, from the wb rows
    {
      const float4 t0 = lds.wb.r[0][lane], t1 = lds.wb.r[1][lane];
      tau[0] = t0.x; tau[1] = t0.y; tau[2] = t0.z; tau[3] = t0.w; tau[4] = t1.x; tau[5] = t1.y;
    }
    if (active) {
      B.contact_vimp[(size_t)n * NVIMP + vimp_base(leg)] = vi_b;
#pragma unroll
      for (int k = 0; k < NLEG; ++k) B.torques[n * 12 + j0 + k] = tau[k];
    }
    if constexpr (FUSED)
#pragma unroll
      for (int k = 0; k < NLEG; ++k) lds.fr[F_TQ + j0 + k][e] = tau[k];
    float vl, vr;
    halves(vi_b, vl, vr);  // the base box's two halves' end-of-step episodes (leg-0 lanes report the whole box)
    __syncthreads();  // R1: the end-of-step state published
    V3<float> fb = v3<float>(0.0f, 0.0f, 0.0f);
    {
      BaseState<float> sb;
      float q[NLEG], qd[NLEG];
      read_state_rows(lds.st, lane, sb, q, qd);
      if (leg == 0) {
      BaseFrame<float> F;
      base_frame(sb, F);
      const float vt0 = restitution_target(M, eg, vl), vt1 = restitution_target(M, eg, vr);
      fb = body_contact_force(M, T, 0, F.R0, v3<float>(0, 0, 0), F.abs, F.V0, mu, vt0 > vt1 ? vt0 : vt1);
      }
    }
    __syncthreads();  // RB: the report's parts in LDS
    if (leg == 0) {
      if (active) {
        float* cf = B.contact_forces + (size_t)n * 39;
        cf[0] = fb.x; cf[1] = fb.y; cf[2] = fb.z;
      }
      if constexpr (FUSED) { lds.fr[F_CFB][e] = fb.x; lds.fr[F_CFB + 1][e] = fb.y; lds.fr[F_CFB + 2][e] = fb.z; }
    }
    T1_PROF_MARK(10);
    if constexpr (FUSED) __syncthreads();  // the epilogue barrier
    T1_CLOCK_WAVE_END();
    T1_PROF_END();
    return;
  }

  if (role != 0) {
    // ======== the term roles W1-W3, W5-W7
    const int wi = shift6_index(role);
    const float mu = 0.5f * (B.friction[n] + M.ground_friction);  // robot shape vs ground (PhysX average)
    const float mu_self = B.friction[n];                          // robot shape vs robot shape
    const float eg = ground_restitution(M, B.restitution[n]);
    // the epilogue's inputs the step does not change, staged by W4-W7 before their first substep
    if (FUSED && wave >= 4) stage_epilogue_inputs<NE6, 256>(B, N, (int)r0, (int)threadIdx.x - 256, lds.epi);
    const int bsh = 1 + 6 * leg + K_SHANK, bft = 1 + 6 * leg + K_FOOT;
    const int half = role >= 4 ? 1 : 0;  // roles 2 / 3: points 0-3, 6 / 7: points 4-7
    // each role its own substep loop (the register allocation of one role's loop does not carry the others' values)
    if (role == 1) {
      // ---- W1: RNEA bias terms of the leg
      LegParams<float> PL;
      load_leg_params(M, B, n, j0, PL);
      ShiftHold hold;  // the pipelined history shift's loads in flight (its own live range per role loop)
      if (wi >= 0) shp_issue_slice(S, r0, r1, 0, nsub, wi, lane, hold);
      for (int sub = 0; sub < nsub; ++sub) {
        T1_PROF_MARK(4);
        D6_S1(sub + 1);  // S1
        T1_PROF_MARK(1);
        BaseState<float> sb;
        float q[NLEG], qd[NLEG];
        read_state_rows(lds.st, lane, sb, q, qd);
        BaseFrame<float> F;
        base_frame(sb, F);
        const float zero6[NLEG] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
        float rg[NLEG], G[6], v[R_N];
        leg_bias_rhs(M, PL, F, q, qd, zero6, leg, dt, rg, G);  // -S_k . sum g (W0 adds dt tau_k)
#pragma unroll
        for (int k = 0; k < NLEG; ++k) v[R_RG + k] = rg[k];
#pragma unroll
        for (int i = 0; i < 6; ++i) v[R_G + i] = G[i];
        put4(lds.w1, lane, v);
        if (wi >= 0 && ((SHIFT6_PRE_MASK >> role) & 1)) {  // the slice before S2 (T1_D6_SHIFT_PRE_MASK)
          shp_commit_slice(S, r0, r1, sub, nsub, wi, lane, hold);
          shp_issue_slice(S, r0, r1, sub + 1, nsub, wi, lane, hold);
        }
        T1_PROF_MARK(2);
        __syncthreads();  // S2
        T1_PROF_MARK(3);
        if (wi >= 0 && !((SHIFT6_PRE_MASK >> role) & 1)) {  // slice sub (its loads issued a substep ago), then
          shp_commit_slice(S, r0, r1, sub, nsub, wi, lane, hold);  // slice sub + 1's loads
          shp_issue_slice(S, r0, r1, sub + 1, nsub, wi, lane, hold);
        }
      }
    } else if (role == 5) {
      // ---- W5: self-contact terms of the shank and foot
      ShiftHold hold;  // the pipelined history shift's loads in flight (its own live range per role loop)
      if (wi >= 0) shp_issue_slice(S, r0, r1, 0, nsub, wi, lane, hold);
      for (int sub = 0; sub < nsub; ++sub) {
        T1_PROF_MARK(4);
        D6_S1(sub + 1);  // S1
        T1_PROF_MARK(1);
        BaseState<float> sb;
        float q[NLEG], qd[NLEG];
        read_state_rows(lds.st, lane, sb, q, qd);
        BaseFrame<float> F;
        base_frame(sb, F);
        BodyKin<float> Ko[2];
        leg_body_kinematics(M, F, q, qd, leg, Ko);
        Sym6<float> Cs[2];
        float cs[2][6];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          sym_zero(Cs[i]);
#pragma unroll
          for (int j = 0; j < 6; ++j) cs[i][j] = 0.0f;
        }
        if (M.self_collisions) {
          SelfBody<float> O[2], X[2];
          self_bodies(M, leg, Ko, O, X);
          self_terms_bodies(M, leg, O, X, mu_self, dt, Cs, cs);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          float v[XCH];
          sym_pack(Cs[i], cs[i], v);
          put4(lds.wc[WC_SSH + i], lane, v);
        }
        if (wi >= 0 && ((SHIFT6_PRE_MASK >> role) & 1)) {  // the slice before S2 (T1_D6_SHIFT_PRE_MASK)
          shp_commit_slice(S, r0, r1, sub, nsub, wi, lane, hold);
          shp_issue_slice(S, r0, r1, sub + 1, nsub, wi, lane, hold);
        }
        T1_PROF_MARK(2);
        __syncthreads();  // S2
        T1_PROF_MARK(3);
        if (wi >= 0 && !((SHIFT6_PRE_MASK >> role) & 1)) {  // slice sub (its loads issued a substep ago), then
          shp_commit_slice(S, r0, r1, sub, nsub, wi, lane, hold);  // slice sub + 1's loads
          shp_issue_slice(S, r0, r1, sub + 1, nsub, wi, lane, hold);
        }
      }
    } else {
      // ---- W2 / W6: shank terrain, W3 / W7: foot terrain (one half of the body's points each); W6 also records the
      // sensor-lag samples and the substep log from the state it reads at S1
      const bool shank = role == 2 || role == 6;
      int s_dof = 9 - B.dof_lag_timestep[n] % 10;
#ifdef T1_MUTANT_CAPTURE  // mutation check of tests/test_gpu_product_parity.py only (tools/gpu): capture a substep early
      s_dof = s_dof > 0 ? s_dof - 1 : 0;
#endif
      const int s_imu = 9 - B.imu_lag_timestep[n] % 10;

      const int slot = (shank ? WC_SHA : WC_FTA) + half;
      const int b = shank ? bsh : bft;
      const int c0 = M.contact_start[b] + half * (T1_POINTS_PER_BODY / 2);
      ShiftHold hold;  // the pipelined history shift's loads in flight (its own live range per role loop)
      if (wi >= 0) shp_issue_slice(S, r0, r1, 0, nsub, wi, lane, hold);
      for (int sub = 0; sub < nsub; ++sub) {
        T1_PROF_MARK(4);
        D6_S1(sub + 1);  // S1
        T1_PROF_MARK(1);
        BaseState<float> sb;
        float q[NLEG], qd[NLEG];
        read_state_rows(lds.st, lane, sb, q, qd);
        if (role == 6 && sub > 0)
          record_substep(M, lds.pb[lane], LG, lds, sub - 1, s_dof, s_imu, N, n, j0, leg, lane, active, sb, q, qd);
        BaseFrame<float> F;
        base_frame(sb, F);
        BodyKin<float> Ko[2];
        leg_body_kinematics(M, F, q, qd, leg, Ko);
        Sym6<float> Cc;
        float cc[6] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
        sym_zero(Cc);
        float amax;
        if (shank) {
          const float vtg = restitution_target(M, eg, lds.vish[lane]);
          contact_half<HF, true>(M, T, c0, Ko[0], F, b, mu, vtg, dt, Cc, cc, amax);
        } else {
          const float vtg = restitution_target(M, eg, lds.vift[lane]);
          contact_half<HF, false>(M, T, c0, Ko[1], F, b, mu, vtg, dt, Cc, cc, amax);
        }
        float v[XCH];
        sym_pack(Cc, cc, v);
        put4(lds.wc[slot], lane, v);
        lds.amx[slot][lane] = amax;
        if (wi >= 0 && ((SHIFT6_PRE_MASK >> role) & 1)) {  // the slice before S2 (T1_D6_SHIFT_PRE_MASK)
          shp_commit_slice(S, r0, r1, sub, nsub, wi, lane, hold);
          shp_issue_slice(S, r0, r1, sub + 1, nsub, wi, lane, hold);
        }
        T1_PROF_MARK(2);
        __syncthreads();  // S2
        T1_PROF_MARK(3);
        if (wi >= 0 && !((SHIFT6_PRE_MASK >> role) & 1)) {  // slice sub (its loads issued a substep ago), then
          shp_commit_slice(S, r0, r1, sub, nsub, wi, lane, hold);  // slice sub + 1's loads
          shp_issue_slice(S, r0, r1, sub + 1, nsub, wi, lane, hold);
        }
      }
    }
    T1_PROF_MARK(4);
    if (wi >= 0) __builtin_amdgcn_s_waitcnt(0);  // the shift's stores complete before the epilogue zeroes reset rows
    T1_PROF_MARK(8);
    __syncthreads();  // R1: the end-of-step state and episodes published
    T1_PROF_MARK(9);
    {  // the contact-force report from the end-of-step state: W2 the shank's terrain force, W3 the foot's, W5 their
       // self-contact forces; W6 sums and stores the shank / foot rows after RB (the base box: W4)
      if (role == 2 || role == 3 || role == 5) {
        BaseState<float> sb;
        float q[NLEG], qd[NLEG];
        read_state_rows(lds.st, lane, sb, q, qd);
        BaseFrame<float> F;
        base_frame(sb, F);
        BodyKin<float> Ko[2];
        leg_body_kinematics(M, F, q, qd, leg, Ko);
        if (role == 5) {
          V3<float> fself[2] = {v3<float>(0.0f, 0.0f, 0.0f), v3<float>(0.0f, 0.0f, 0.0f)};
          if (M.self_collisions) {
            SelfBody<float> O[2], X[2];
            self_bodies(M, leg, Ko, O, X);
            self_forces_bodies(M, leg, O, X, mu_self, fself);
          }
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            lds.rsf[s][0][lane] = fself[s].x; lds.rsf[s][1][lane] = fself[s].y; lds.rsf[s][2][lane] = fself[s].z;
          }
        } else {
          const int s = role == 2 ? 0 : 1;
          const int b = s == 0 ? bsh : bft;
          const float vt = restitution_target(M, eg, s == 0 ? lds.vish[lane] : lds.vift[lane]);
          const V3<float> f = body_contact_force(M, T, b, Ko[s].Rb, Ko[s].p, F.abs, Ko[s].V, mu, vt);
          lds.rtf[s][0][lane] = f.x; lds.rtf[s][1][lane] = f.y; lds.rtf[s][2][lane] = f.z;
        }
      }
      T1_PROF_MARK(10);
      if (role == 6) {  // the last substep's state (published before R1): its log row, then the lag samples' stores
        int s_dof = 9 - B.dof_lag_timestep[n] % 10;
#ifdef T1_MUTANT_CAPTURE
        s_dof = s_dof > 0 ? s_dof - 1 : 0;
#endif
        const int s_imu = 9 - B.imu_lag_timestep[n] % 10;
        BaseState<float> sb;
        float q[NLEG], qd[NLEG];
        read_state_rows(lds.st, lane, sb, q, qd);
        record_substep(M, lds.pb[lane], LG, lds, nsub - 1, s_dof, s_imu, N, n, j0, leg, lane, active, sb, q, qd);
        if (active) {  // the sensor-lag samples into the step's ring slots
          float* const dof_dst = B.dof_hist + ((size_t)n * 4 + (ctr & 3u)) * 24;
          float* const imu_dst = B.imu_hist + ((size_t)n * 2 + (ctr & 1u)) * 8;
          if (s_dof < nsub) {
#pragma unroll
            for (int k = 0; k < NLEG; ++k) {
              dof_dst[j0 + k] = lds.cap[k][lane];
              dof_dst[12 + j0 + k] = lds.cap[NLEG + k][lane];
            }
          }
          if (leg == 0 && s_imu < nsub) {
            const float quat[4] = {lds.cap[2 * NLEG][lane], lds.cap[2 * NLEG + 1][lane], lds.cap[2 * NLEG + 2][lane],
                                   lds.cap[2 * NLEG + 3][lane]};
            const float w[3] = {lds.cap[2 * NLEG + 4][lane], lds.cap[2 * NLEG + 5][lane], lds.cap[2 * NLEG + 6][lane]};
            capture_imu(quat, w, imu_dst);
          }
        }
      }
      __syncthreads();  // RB: the report's parts in LDS
      T1_PROF_MARK(11);
      if (role == 6) {
        float* cf = B.contact_forces + (size_t)n * 39;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int b = s == 0 ? bsh : bft;
          const float f[3] = {lds.rtf[s][0][lane] + lds.rsf[s][0][lane], lds.rtf[s][1][lane] + lds.rsf[s][1][lane],
                              lds.rtf[s][2][lane] + lds.rsf[s][2][lane]};
          if (active) { cf[b * 3 + 0] = f[0]; cf[b * 3 + 1] = f[1]; cf[b * 3 + 2] = f[2]; }
          if (FUSED && s == 1) {
            const int r = leg == 0 ? F_C0 : F_C1;
            lds.fr[r][e] = f[0]; lds.fr[r + 1][e] = f[1]; lds.fr[r + 2][e] = f[2];
          }
        }
      }
    }
    if constexpr (FUSED) {
      __syncthreads();  // the epilogue barrier: every output of the workgroup is in LDS / memory
      T1_PROF_MARK(12);
#ifndef T1_WHATIF_D6_EPI_SKIP  // timing-only what-if builds: bit r set = role r skips its epilogue part
#define T1_WHATIF_D6_EPI_SKIP 0
#endif
      if ((T1_WHATIF_D6_EPI_SKIP >> role) & 1) {
      } else if (role == 1)
        fused_epilogue_staged<POST_A_STATE, NE6, true>(M, C, B, A, S, FA, dyn_blocks, lane, lds.epi, lds.fr, lds.act,
                                                       lds.act + NLEG);
      else if (role == 2)
        fused_epilogue_obs<POST_OBS_PRIV, NE6>(M, C, B, A, lane, lds.epi, lds.fr, lds.act, lds.act + NLEG);
      else if (role == 3)
        fused_epilogue_obs<POST_OBS_ACTOR, NE6>(M, C, B, A, lane, lds.epi, lds.fr, lds.act, lds.act + NLEG);
      T1_PROF_MARK(15);
    }
    T1_CLOCK_WAVE_END();
    T1_PROF_END();
    return;
  }

  // ======== W0: core -- pose chain + contact-free CRBA backward pass; after S2 fold-in, elimination, base system,
  // integration; owns the joint state and the restitution episodes of the shank and foot
  BaseParams<float>& PB = lds.pb[lane];
  LegParams<float>& PL = lds.pl[lane];
  {  // the state is held in LDS (lds.st, which W0 alone writes), not in registers across the substep loop
    BaseState<float> sb;
    float q[NLEG], qd[NLEG];
    BaseParams<float> pb;
    LegParams<float> pl;
    load_base_params(M, B, n, pb);
    load_leg_params(M, B, n, j0, pl);
    load_base_state(M, pb, B.root_states + (size_t)n * 13, sb);
    PB = pb;
    PL = pl;
#pragma unroll
    for (int k = 0; k < NLEG; ++k) {
      q[k] = B.dof_state[n * 24 + 2 * (j0 + k)];
      qd[k] = B.dof_state[n * 24 + 2 * (j0 + k) + 1];
    }
    float v[Q_N];
    state_pack(sb, q, qd, v);
    put4(lds.st, lane, v);
  }
  float vi_ft = B.contact_vimp[(size_t)n * NVIMP + vimp_foot(leg)];
  float vi_sh = B.contact_vimp[(size_t)n * NVIMP + vimp_shank(leg)];
  lds.vift[lane] = vi_ft;
  lds.vish[lane] = vi_sh;
  T1_PROF_MARK(0);
#ifdef T1_D6_S1_FLAG
  s1_signal(&lds.s1flag, 1);  // the first substep's state (and the episodes) published
#endif
  for (int sub = 0; sub < nsub; ++sub) {
#ifndef T1_D6_S1_FLAG
    {
      T1_CLOCK_WAIT_BEGIN();
      __syncthreads();  // S1: the substep state published
      T1_CLOCK_WAIT_END(1);
    }
#endif
    T1_PROF_MARK(1);
    // -DT1_D6_LAUNDER (A/B): the lane and leg through an empty asm each substep, so the lane- and leg-indexed LDS
    // addresses are formed in the loop instead of hoisted and spilled: no scratch reloads in the loop, yet measured
    // 0.5-1% slower (r05ab2, r05o2)
    int lane_s = lane, leg_s = leg;
#ifdef T1_D6_LAUNDER
    asm volatile("" : "+v"(lane_s), "+v"(leg_s));
#endif
    const DynModel& M = model_in_loop(lds.model);
    LegBlock<float> lb;
    Sym6<float> Ab;
    {
      BaseState<float> sb;
      float q[NLEG], qd[NLEG];
      read_state_rows(lds.st, lane_s, sb, q, qd);
      const M3<float> R0 = quat_to_mat(sb.quat[0], sb.quat[1], sb.quat[2], sb.quat[3]);  // base_frame's F.R0
      LegFK<float> fk;
      leg_fk_chain(M, R0, q, leg_s, fk);
      float Sj[NLEG][6];
      sym_zero(Ab);
      leg_backward_crba(M, PL, q, qd, leg_s, dt, fk, Sj, lb, Ab);
#pragma unroll
      for (int k = 0; k < NLEG; ++k) {  // the joint subspaces to LDS for the fold-in (registers at its peak)
        lds.sj.r[k][0][lane_s] = make_float4(Sj[k][0], Sj[k][1], Sj[k][2], Sj[k][3]);
        lds.sj.r[k][1][lane_s] = make_float4(Sj[k][4], Sj[k][5], 0.0f, 0.0f);
      }
    }
    T1_PROF_MARK(2);
    {
      T1_CLOCK_WAIT_BEGIN();
      __syncthreads();  // S2: the terms published
      T1_CLOCK_WAIT_END(2);
    }
    T1_PROF_MARK(3);
    {  // the episodes of the shank and foot from the two halves of their points
      vi_sh = restitution_episode(vi_sh, fmaxf(lds.amx[WC_SHA][lane_s], lds.amx[WC_SHB][lane_s]));
      vi_ft = restitution_episode(vi_ft, fmaxf(lds.amx[WC_FTA][lane_s], lds.amx[WC_FTB][lane_s]));
      lds.vish[lane_s] = vi_sh;  // W2 / W6 read it after the next S1
      lds.vift[lane_s] = vi_ft;  // W3 / W7
    }
    float g6[6] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    {
      float rg[NLEG];  // dt tau_k (W4's torques, the first two rows of wb) + the bias part (W1)
      const float4 t0 = lds.wb.r[0][lane_s], t1 = lds.wb.r[1][lane_s];
      const float4 g0 = lds.w1.r[0][lane_s], g1 = lds.w1.r[1][lane_s];
      const float tv[NLEG] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y}, gv[NLEG] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y};
      static_assert(WB_TAU == 0 && R_RG == 0, "the torques and the bias rhs lead their rows");
#pragma unroll
      for (int k = 0; k < NLEG; ++k) rg[k] = dt * tv[k] + gv[k];
#ifndef T1_WHATIF_D6_NO_FOLDIN  // timing-only what-if build: the contact / bias terms not folded in
      leg_apply_terms_rows<K_SHANK, K_FOOT>(lds.wc, lds.w1, rg, lds.sj, lane_s, lb, Ab, g6);
#else
      for (int k = 0; k < NLEG; ++k) lb.rhs[k] += rg[k];
#endif
    }
    T1_PROF_MARK(5);
    float rb[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) rb[i] = -g6[i];
    eliminate_leg(lb, Ab, rb);
    T1_PROF_MARK(6);
    // the base system: (base block + both base-box halves, W4) + the left leg + the right leg, in every lane
    Sym6<float> Ac;
    float r[6];
    {
      float v[WB_N];
      get4(lds.wb, lane_s, v);
#pragma unroll
      for (int i = 0; i < 21; ++i) Ac.a[i] = v[WB_AC + i];
#pragma unroll
      for (int i = 0; i < 6; ++i) r[i] = v[WB_R + i];
    }
#pragma unroll
    for (int i = 0; i < 21; ++i) {
      float l, rr;
      halves(Ab.a[i], l, rr);
      Ac.a[i] = (Ac.a[i] + l) + rr;
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      float l, rr;
      halves(rb[i], l, rr);
      r[i] = (r[i] + l) + rr;
    }
    solve_base(Ac, r);
    float dq[NLEG];
    backsub_leg(lb, r, dq);
    BaseState<float> sb;
    float q[NLEG], qd[NLEG];
    read_state_rows(lds.st, lane_s, sb, q, qd);
    integrate_base(sb, r, dt);
    integrate_leg(M, leg_s, q, qd, dq, dt);
    float v[Q_N];
    state_pack(sb, q, qd, v);
    put4(lds.st, lane_s, v);  // the roles read the previous state before S2; after the last substep: the report's
#ifdef T1_D6_S1_FLAG
    s1_signal(&lds.s1flag, sub + 2);
#endif
    T1_PROF_MARK(7);
  }
  T1_CLOCK_LOOP_END();
  BaseState<float> sb;
  float q[NLEG], qd[NLEG];
  read_state_rows(lds.st, lane, sb, q, qd);
  if (active) {
    B.contact_vimp[(size_t)n * NVIMP + vimp_foot(leg)] = vi_ft;
    B.contact_vimp[(size_t)n * NVIMP + vimp_shank(leg)] = vi_sh;
#pragma unroll
    for (int k = 0; k < NLEG; ++k) {
      B.dof_state[n * 24 + 2 * (j0 + k)] = q[k];
      B.dof_state[n * 24 + 2 * (j0 + k) + 1] = qd[k];
    }
  }
  float (*FR)[NE6] = FUSED ? lds.fr : nullptr;
  if constexpr (FUSED) {
#pragma unroll
    for (int k = 0; k < NLEG; ++k) {
      lds.fr[F_DOF + 2 * (j0 + k)][e] = q[k];
      lds.fr[F_DOF + 2 * (j0 + k) + 1][e] = qd[k];
    }
  }
  T1_PROF_MARK(8);
  __syncthreads();  // R1: the end-of-step state published (the report's contact forces meanwhile)
  T1_PROF_MARK(9);
  {
    BaseFrame<float> F;
    base_frame(sb, F);
    leg_report_rigid<NE6>(M, B, PB, sb, F, q, qd, n, leg, active, e, FR);
  }
  T1_PROF_MARK(10);
  __syncthreads();  // RB: the contact-force report's parts in LDS
  T1_PROF_MARK(11);
  if constexpr (FUSED) {
    __syncthreads();  // the epilogue barrier: every output of the workgroup is in LDS / memory
    T1_PROF_MARK(12);
    fused_epilogue_staged<POST_A_REWARDS, NE6, true>(M, C, B, A, S, FA, dyn_blocks, lane, lds.epi, lds.fr, lds.act,
                                                     lds.act + NLEG);
  }
  T1_CLOCK_END();
  T1_PROF_END();
}

#ifdef T1_PROBE_SIMD
extern "C" int t1env_debug_simd6(unsigned* out, int blocks) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_t1_simd6), sizeof(unsigned) * 8 * (size_t)blocks);
}
#endif

#ifdef T1_PROBE_CLOCK
// probe build only: {cycles, constant-clock ticks, workgroup count} summed since the last reset (reset != 0: zeroed after
// the read)
extern "C" int t1env_debug_wgtime6(unsigned long long* out, int blocks) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_t1_wgtime6), sizeof(unsigned long long) * 4 * (size_t)blocks);
}
extern "C" int t1env_debug_wgsum6(unsigned long long* out, int blocks, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_t1_wgsum6), sizeof(unsigned long long) * 3 * (size_t)blocks);
  if (e == hipSuccess && reset) {
    static unsigned long long zero[4096][3] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_t1_wgsum6), zero, sizeof(zero));
  }
  return (int)e;
}
extern "C" int t1env_debug_clock6(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_t1_clock6), sizeof(g_t1_clock6));
  if (e == hipSuccess && reset) {
    static const unsigned long long zero[4] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_t1_clock6), zero, sizeof(zero));
  }
  return (int)e;
}
#endif

#ifdef T1_PHASE_PROF
// profiling build only: summed clock deltas per [wave][bucket] since the last reset
extern "C" int t1env_debug_phase_cycles6(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_t1_prof6), sizeof(g_t1_prof6));
  if (e == hipSuccess && reset) {
    static const unsigned long long zero[T1_PROF_WAVES6][T1_NPROF6] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_t1_prof6), zero, sizeof(zero));
  }
  return (int)e;
}
#endif

int t1_launch_dyn6(const DynModel* d_model, const t1env_config* d_cfg, const t1env_buffers& B, const Terrain& T,
                   const float* actions, const t1env_step_args& A, int num_envs, const ShiftArgs& S,
                   const FusedArgs* fused, hipStream_t s, const SubLog* log) {
  const int blocks = (num_envs + NE6 - 1) / NE6;
  const FusedArgs FA = fused ? *fused : FusedArgs{};
  const SubLog LG = log ? *log : SubLog{};
  const bool hf = T.type != 0;
  if (log && !fused) return (int)hipErrorInvalidValue;  // the substep log: fused steps only (the caller checks)
#define T1_LAUNCH6(HF, FU) \
  hipLaunchKernelGGL((k_dyn6<HF, FU>), dim3(blocks), dim3(D6_BLOCK), 0, s, d_model, d_cfg, B, T, actions, A, S, blocks, FA, LG)
  if (fused) { if (hf) T1_LAUNCH6(true, true); else T1_LAUNCH6(false, true); }
  else { if (hf) T1_LAUNCH6(true, false); else T1_LAUNCH6(false, false); }
#undef T1_LAUNCH6
  return (int)hipGetLastError();
}
