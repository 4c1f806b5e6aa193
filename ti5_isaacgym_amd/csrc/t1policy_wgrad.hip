// The PPO update's Linear weight and bias gradients under the opt-in bf16 update (include/t1policy.h,
// t1policy_linear_wgrad_bf16): gW = gy^T x and gb = sum_r gy[r] for a batch of rows, in one MFMA kernel plus one
// fixed-order reduction -- what loss.backward() computes for every nn.Linear of the policy (dh_ppo.py:180,
// actor_critic_dh.py:45-111), at the update's 49,152-row minibatch.
//
// The build's path before this (dh_policy.wgrad_splitk + bias_grad): a hipBLASLt strided-batched GEMM over 24 slices
// of 2,048 rows, the slices summed by t1policy_slice_sum, and torch's dim-0 sum for the bias -- three launches per
// layer and 10 ms of device time per update (bmm 5.4 ms + sums 4.7 ms, profiles/r04q_ppo_update_profile_bf16_eager.txt)
// for ~0.7 TFLOP.
//
// Both operands are row-major with the REDUCTION (the batch row) as their slow index, so the MFMA fragments -- a lane
// holds 8 consecutive k of one output row / column -- are columns of the staged tiles: each 32-row chunk of gy and x is
// staged into LDS row-major as loaded (coalesced dword loads, realigned for an odd width; three chunks of loads in
// flight through a register ring), and the fragments come
// back with ds_read_b64_tr_b16 (the gfx950 transposing LDS read: a 16-lane group reads 4 rows x 16 columns and gets
// the columns in its lanes).  A workgroup owns a 128 x 128 output tile and a slice of rows; its four waves own 64 x 64
// quarters (2 x 2 v_mfma_f32_32x32x16_bf16 accumulators).  The bias sum rides on the A fragments of the n-tile-0
// workgroups.  Partials go to a workspace [slice][M x N | M]; k_wgrad_reduce sums the slices in a fixed tree, so the
// result is deterministic (eager and graph-replayed updates stay bit-identical).  Products of bf16 operands are
// exact in fp32; the sums are fp32.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

namespace {

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef short s4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr int WG_T = 128;             // output tile (m and n)
constexpr int WG_ROWS = 32;           // rows per staged chunk (two k-steps of 16)
constexpr int WG_PITCH = WG_T + 32;   // LDS row pitch in 16-bit elements: 320 B, rows 16 banks apart (conflict-free
                                      // transposed reads: a 32-lane half's two groups x 4 rows cover the 64 banks once)
constexpr int WG_IMG = WG_ROWS * WG_PITCH;  // one staged operand chunk (elements)
constexpr int WG_MIN_ROWS = 256;      // rows per slice at least

__device__ __forceinline__ float bf16_float(uint16_t b) { return __uint_as_float((uint32_t)b << 16); }

// a 32-row chunk of columns [c0, c0 + 128) of a (rows, W) bf16 matrix: thread t loads the column pair 2 (t & 63) of
// rows r0 + (t >> 6) + 4 i.  W even: the pair is an aligned dword.  W odd (c0, r0 even): a row starts at an element of
// the row's parity, the wave's parity: even rows take the aligned dword, odd rows the two aligned dwords around the
// pair, realigned by a 16-bit shift.  Every load is issued unconditionally at a clamped in-matrix index, and the raw
// dwords stay in the register ring until the chunk is staged (wg_store applies the realignment and zeroes the pairs past
// the slice end or the width): a conditional load, or a select right behind the load, makes the compiler wait for it
// there and drains the ring.
template <bool PAIR> struct WgStage {
  uint32_t lo[8];
  uint32_t hi[PAIR ? 1 : 8];
};
template <bool PAIR>
__device__ __forceinline__ void wg_load(const uint16_t* __restrict__ z, int W, int c0, int r0, int r1, int rows, int t,
                                        WgStage<PAIR>& v) {
  const int col = c0 + 2 * (t & 63);
  const int colc = col < W ? col : (W - 1) & ~1;
  const uint32_t* zw = reinterpret_cast<const uint32_t*>(z);
  const size_t last = ((size_t)rows * W - 1) >> 1;  // the dword holding the matrix's last element
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = r0 + (t >> 6) + 4 * i;
    const size_t e = (size_t)(r < r1 ? r : r1 - 1) * W + colc;
    v.lo[i] = zw[e >> 1];
    if constexpr (!PAIR) {
      const size_t ih = (e >> 1) + 1;
      v.hi[i] = zw[ih < last ? ih : last];
    }
  }
}

template <bool PAIR>
__device__ __forceinline__ void wg_store(uint32_t* img, int W, int c0, int r0, int r1, int t, const WgStage<PAIR>& v) {
  const bool c_ok = c0 + 2 * (t & 63) < W;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const bool ok = c_ok && r0 + (t >> 6) + 4 * i < r1;
    uint32_t u = v.lo[i];
    if constexpr (!PAIR) u = ((t >> 6) & 1) ? (u >> 16) | (v.hi[i] << 16) : u;
    img[((t >> 6) + 4 * i) * (WG_PITCH / 2) + (t & 63)] = ok ? u : 0u;
  }
}

// the 32 x 16 (A) or 16 x 32 (B) fragment of k-step ks for columns [col0, col0 + 32) of a staged chunk: lane
// (r = l & 31, h = l >> 5) gets rows 16 ks + 8 h + j, j = 0 .. 7, of column col0 + r -- two transposed reads of
// 4 rows each (lane 4 q + p of a 16-lane group addresses row q, columns 4 p .. 4 p + 3 of its 16-column block)
__device__ __forceinline__ bf8 wg_frag(const uint16_t* img, int ks, int col0, int lane) {
  const int g = lane >> 4, i = lane & 15, h = g >> 1;
  const int row = 16 * ks + 8 * h + (i >> 2);
  const int col = col0 + 16 * (g & 1) + 4 * (i & 3);
  typedef __attribute__((address_space(3))) s4 lds_s4;
  const uint16_t* p = img + row * WG_PITCH + col;
  const s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(p));
  const s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(p + 4 * WG_PITCH));
  typedef short s8 __attribute__((ext_vector_type(8)));
  const s8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf8, v);
}

// grid: x = output tile (tm + tiles_m tn), y = slice of rows_per_slice rows.  part: [slice][M][N], bpart: [slice][M]
template <bool GY_PAIR, bool X_PAIR>
__global__ __launch_bounds__(256, 2) void k_linear_wgrad_bf16(const uint16_t* __restrict__ gy,
                                                              const uint16_t* __restrict__ x, int rows, int M, int N,
                                                              int tiles_m, int rows_per_slice,
                                                              float* __restrict__ part, float* __restrict__ bpart) {
  __shared__ __attribute__((aligned(16))) uint16_t IMG[2][2][WG_IMG];  // [buffer][gy, x]
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, h = lane >> 5;
  const int wm = wave & 1, wn = wave >> 1;
  const int tm = blockIdx.x % tiles_m, tn = blockIdx.x / tiles_m, s = blockIdx.y;
  const int m0 = WG_T * tm, n0 = WG_T * tn;
  const int r0 = s * rows_per_slice;
  const int r1 = r0 + rows_per_slice < rows ? r0 + rows_per_slice : rows;
  // this wave's 32-wide blocks that hold outputs (wave-uniform)
  const int m_rem = M - (m0 + 64 * wm), n_rem = N - (n0 + 64 * wn);
  const int mb_n = m_rem <= 0 ? 0 : (m_rem > 32 ? 2 : 1), nb_n = n_rem <= 0 ? 0 : (n_rem > 32 ? 2 : 1);
  const bool bias = bpart != nullptr && tn == 0 && wn == 0;  // (nb_n >= 1 there)
  f16v acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.0f;
  float bsum[2] = {0.0f, 0.0f};
  // three chunks of loads in flight: register slots 0, 1, 2 hold chunks c, c + 1, c + 2; a slot is refilled with chunk
  // c + 3 as soon as it is staged into LDS (two LDS buffers, one barrier per chunk)
  WgStage<GY_PAIR> vg[3];
  WgStage<X_PAIR> vx[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    wg_load<GY_PAIR>(gy, M, m0, r0 + k * WG_ROWS, r1, rows, t, vg[k]);
    wg_load<X_PAIR>(x, N, n0, r0 + k * WG_ROWS, r1, rows, t, vx[k]);
    __builtin_amdgcn_sched_barrier(0);  // slot order = issue order (the waits count on it)
  }
  int buf = 0;
  auto chunk = [&](WgStage<GY_PAIR>& rg, WgStage<X_PAIR>& rx, int c) {
    wg_store<GY_PAIR>(reinterpret_cast<uint32_t*>(IMG[buf][0]), M, m0, c, r1, t, rg);
    wg_store<X_PAIR>(reinterpret_cast<uint32_t*>(IMG[buf][1]), N, n0, c, r1, t, rx);
    // refill unconditionally (past the slice end: the slice's last row again, never stored), so the wait before
    // each store counts only this slot's loads
    wg_load<GY_PAIR>(gy, M, m0, c + 3 * WG_ROWS, r1, rows, t, rg);
    wg_load<X_PAIR>(x, N, n0, c + 3 * WG_ROWS, r1, rows, t, rx);
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();  // staged; double-buffered, so the chunk before last's readers are done
    if (mb_n > 0 && nb_n > 0) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf8 fa[2], fb[2];
#pragma unroll
        for (int a = 0; a < 2; ++a) fa[a] = wg_frag(IMG[buf][0], ks, 64 * wm + 32 * a, lane);
#pragma unroll
        for (int b = 0; b < 2; ++b) fb[b] = wg_frag(IMG[buf][1], ks, 64 * wn + 32 * b, lane);
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          if (a >= mb_n) break;
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            if (b >= nb_n) break;
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a], fb[b], acc[a][b], 0, 0, 0);
          }
          if (bias) {
#pragma unroll
            for (int j = 0; j < 8; ++j) bsum[a] += (float)fa[a][j];
          }
        }
      }
    }
    buf ^= 1;
  };
  for (int c = r0; c < r1; c += 3 * WG_ROWS) {
    chunk(vg[0], vx[0], c);
    if (c + WG_ROWS >= r1) break;
    chunk(vg[1], vx[1], c + WG_ROWS);
    if (c + 2 * WG_ROWS >= r1) break;
    chunk(vg[2], vx[2], c + 2 * WG_ROWS);
  }
  // C/D: column n = lane & 31, row m = (r & 3) + 8 (r >> 2) + 4 h
  float* P = part + (size_t)s * M * N;
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    if (a >= mb_n) break;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      if (b >= nb_n) break;
      const int n = n0 + 64 * wn + 32 * b + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + 64 * wm + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m < M && n < N) P[(size_t)m * N + n] = acc[a][b][r];
      }
    }
  }
  if (bias) {
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      if (a >= mb_n) break;
      const float v = bsum[a] + __shfl_xor(bsum[a], 32);  // the two row halves of column m, in a fixed order
      const int m = m0 + 64 * wm + 32 * a + (lane & 31);
      if (h == 0 && m < M) bpart[(size_t)s * M + m] = v;
    }
  }
}

// ---- the fp32 update (the reference's precision, dh_ppo.py:155-182): the same tiles, slices, partials and reduction on
// fp32 gy and x.  A chunk of 32 rows is staged as fp32 rows (pitch 132 words: a fragment read's two 32-lane halves,
// 8 rows apart, cover the 64 banks once); a wave reads each 8-element fragment column with eight ds_read_b32 and splits
// every value into three bf16 parts (v1 = bf16(v), v2 = bf16(v - v1), v3 = bf16(v - v1 - v2): 24+ bits, exact for
// normal fp32), and each 32 x 32 tile takes the six part products down to 2^-16 of |a b| (the three dropped ones are
// below 2^-24): fp32-class sums of exact bf16 products, deterministic as the bf16 kernel's.  The bias sums the fp32 gy.
// 1,158 us per minibatch over the update's 15 layers against 1,340-1,356 for the split-K batched GEMM + slice sum + bias
// sum it replaces (profiles/r06j_*); forming the parts once per staged element (three bf16 images read back by the
// transposing reads) measured the same (1,159 us) and was removed.
constexpr int WG32_PITCH = WG_T + 4;  // fp32 words per staged row
constexpr int WG32_RPT = WG_ROWS / 2;  // rows per thread per chunk (two rows per 256 threads' pass of 128 columns)
struct Wg32Stage {
  float v[WG32_RPT];
};
// thread t loads column c0 + (t & 127) of rows r0 + (t >> 7) + 2 i (coalesced 256-B wave rows), clamped in-matrix and
// issued unconditionally (the store below zeroes what lies outside the slice or the width)
__device__ __forceinline__ void wg32_load(const float* __restrict__ z, int W, int c0, int r0, int r1, int t,
                                          Wg32Stage& v) {
  const int col = c0 + (t & 127);
  const int colc = col < W ? col : W - 1;
#pragma unroll
  for (int i = 0; i < WG32_RPT; ++i) {
    const int r = r0 + (t >> 7) + 2 * i;
    v.v[i] = z[(size_t)(r < r1 ? r : r1 - 1) * W + colc];
  }
}
__device__ __forceinline__ void wg32_store(float* img, int W, int c0, int r0, int r1, int t, const Wg32Stage& v) {
  const bool c_ok = c0 + (t & 127) < W;
#pragma unroll
  for (int i = 0; i < WG32_RPT; ++i) {
    const int rr = (t >> 7) + 2 * i;
    img[rr * WG32_PITCH + (t & 127)] = (c_ok && r0 + rr < r1) ? v.v[i] : 0.0f;
  }
}
struct Bf3f {
  bf8 p[3];
};
// the fragment of k-step ks for column col0 + (lane & 31): rows 16 ks + 8 (lane >> 5) + j, j = 0 .. 7, split in three
__device__ __forceinline__ void wg32_frag(const float* img, int ks, int col0, int lane, Bf3f& f, float* sum) {
  const int row = 16 * ks + 8 * (lane >> 5), col = col0 + (lane & 31);
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = img[(row + j) * WG32_PITCH + col];
  if (sum) {
#pragma unroll
    for (int j = 0; j < 8; ++j) *sum += v[j];
  }
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
__device__ __forceinline__ f16v mfma_bf3f(const Bf3f& a, const Bf3f& b, f16v acc) {  // the smallest products first
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[2], b.p[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[1], b.p[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[0], b.p[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[1], b.p[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[0], b.p[1], acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[0], b.p[0], acc, 0, 0, 0);
}
__global__ __launch_bounds__(256, 2) void k_linear_wgrad_f32(const float* __restrict__ gy, const float* __restrict__ x,
                                                             int rows, int M, int N, int tiles_m, int rows_per_slice,
                                                             float* __restrict__ part, float* __restrict__ bpart) {
  __shared__ __attribute__((aligned(16))) float IMG[2][2][WG_ROWS * WG32_PITCH];  // [buffer][gy, x]
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, h = lane >> 5;
  const int wm = wave & 1, wn = wave >> 1;
  const int tm = blockIdx.x % tiles_m, tn = blockIdx.x / tiles_m, s = blockIdx.y;
  const int m0 = WG_T * tm, n0 = WG_T * tn;
  const int r0 = s * rows_per_slice;
  const int r1 = r0 + rows_per_slice < rows ? r0 + rows_per_slice : rows;
  const int m_rem = M - (m0 + 64 * wm), n_rem = N - (n0 + 64 * wn);
  const int mb_n = m_rem <= 0 ? 0 : (m_rem > 32 ? 2 : 1), nb_n = n_rem <= 0 ? 0 : (n_rem > 32 ? 2 : 1);
  const bool bias = bpart != nullptr && tn == 0 && wn == 0;
  f16v acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.0f;
  float bsum[2] = {0.0f, 0.0f};
  // two chunks of loads in flight (register slots 0, 1), refilled as soon as staged (two LDS buffers, one barrier per
  // chunk)
  Wg32Stage vg[2], vx[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    wg32_load(gy, M, m0, r0 + k * WG_ROWS, r1, t, vg[k]);
    wg32_load(x, N, n0, r0 + k * WG_ROWS, r1, t, vx[k]);
    __builtin_amdgcn_sched_barrier(0);
  }
  int buf = 0;
  auto chunk = [&](Wg32Stage& rg, Wg32Stage& rx, int c) {
    wg32_store(IMG[buf][0], M, m0, c, r1, t, rg);
    wg32_store(IMG[buf][1], N, n0, c, r1, t, rx);
    wg32_load(gy, M, m0, c + 2 * WG_ROWS, r1, t, rg);
    wg32_load(x, N, n0, c + 2 * WG_ROWS, r1, t, rx);
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
    if (mb_n > 0 && nb_n > 0) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        Bf3f fa[2], fb[2];
#pragma unroll
        for (int a = 0; a < 2; ++a)
          wg32_frag(IMG[buf][0], ks, 64 * wm + 32 * a, lane, fa[a], bias && a < mb_n ? &bsum[a] : nullptr);
#pragma unroll
        for (int b = 0; b < 2; ++b) wg32_frag(IMG[buf][1], ks, 64 * wn + 32 * b, lane, fb[b], nullptr);
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          if (a >= mb_n) break;
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            if (b >= nb_n) break;
            acc[a][b] = mfma_bf3f(fa[a], fb[b], acc[a][b]);
          }
        }
      }
    }
    buf ^= 1;
  };
  for (int c = r0; c < r1; c += 2 * WG_ROWS) {
    chunk(vg[0], vx[0], c);
    if (c + WG_ROWS >= r1) break;
    chunk(vg[1], vx[1], c + WG_ROWS);
  }
  float* P = part + (size_t)s * M * N;
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    if (a >= mb_n) break;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      if (b >= nb_n) break;
      const int n = n0 + 64 * wn + 32 * b + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + 64 * wm + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m < M && n < N) P[(size_t)m * N + n] = acc[a][b][r];
      }
    }
  }
  if (bias) {
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      if (a >= mb_n) break;
      const float v = bsum[a] + __shfl_xor(bsum[a], 32);
      const int m = m0 + 64 * wm + 32 * a + (lane & 31);
      if (h == 0 && m < M) bpart[(size_t)s * M + m] = v;
    }
  }
}

// ---- the staged-split form of the fp32 kernel (the default; T1_WGRAD_STAGED=0 selects k_linear_wgrad_f32 above): the
// transpose happens in the registers -- thread t loads column (t & 127) of 8 consecutive rows of a 16-row chunk (each
// wave load is 64 consecutive columns of one row: 256 coalesced bytes), so it holds 8 consecutive k of one output row
// / column, splits them into their three bf16 parts ONCE and stores each part as one ds_write_b128 into [part][col][k]
// images (16 k + 8 pad: 48-B rows, conflict-free b128 stores and reads); the fragments are then one ds_read_b128 per
// part, no VALU between the LDS and the MFMAs.  A chunk's 24 MFMAs run in two halves, the first beside staging the
// next chunk and loading the one after next (a two-slot register ring), the second beside reading the next chunk's
// fragments; one barrier per chunk.  Loads go through buffer descriptors: columns past the width and rows past the
// matrix read 0.  Workgroups of one row slice run on one XCD (their gy and x rows are shared through its L2).  The bias
// sums the staged gy values in a fixed order (8 rows per thread per chunk, then the two row halves).
constexpr int WS_KC = 16, WS_PITCH = 24, WS_IMG = WG_T * WS_PITCH;  // bf16
constexpr int WS_OOB = 0x40000000;
typedef float f8v __attribute__((ext_vector_type(8)));
__device__ __forceinline__ void ws_load(__amdgpu_buffer_rsrc_t rs, int base, int rowb, int k0, f8v& v) {
#pragma unroll
  for (int i = 0; i < 8; ++i)
    v[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, base + (k0 + i) * rowb, 0, 0));
}
__device__ __forceinline__ void ws_split_store(__bf16* img, int col, int g, const f8v& v) {
  bf8 p1, p2, p3;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 h1 = (__bf16)v[j];
    const float r1 = v[j] - (float)h1;
    const __bf16 h2 = (__bf16)r1;
    p1[j] = h1;
    p2[j] = h2;
    p3[j] = (__bf16)(r1 - (float)h2);
  }
  const int o = col * WS_PITCH + 8 * g;
  *reinterpret_cast<bf8*>(img + o) = p1;
  *reinterpret_cast<bf8*>(img + WS_IMG + o) = p2;
  *reinterpret_cast<bf8*>(img + 2 * WS_IMG + o) = p3;
}
__device__ __forceinline__ void ws_frag(const __bf16* img, int col0, int lane, Bf3f& f) {
  const int o = (col0 + (lane & 31)) * WS_PITCH + 8 * (lane >> 5);
#pragma unroll
  for (int p = 0; p < 3; ++p) f.p[p] = *reinterpret_cast<const bf8*>(img + p * WS_IMG + o);
}
struct WsFrags {
  Bf3f a[2], b[2];
};
// grid: 8 x per_xcd workgroups; workgroup i takes unit q = (i mod 8) per_xcd + i / 8 = (slice, tile) with the tile
// fastest
__global__ __launch_bounds__(256, 2) void k_linear_wgrad_f32s(const float* __restrict__ gy, const float* __restrict__ x,
                                                              int ldx, int rows, int M, int N, int tiles_m, int tiles,
                                                              int rows_per_slice, int units, int per_xcd,
                                                              float* __restrict__ part, float* __restrict__ bpart) {
  __shared__ __attribute__((aligned(16))) __bf16 IMG[2][2][3 * WS_IMG];  // [buffer][gy, x][part][col][k]
  const int q = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  if (q >= units) return;  // uniform
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, h = lane >> 5;
  const int wm = wave & 1, wn = wave >> 1;
  const int tile = q % tiles, s = q / tiles;
  const int tm = tile % tiles_m, tn = tile / tiles_m;
  const int m0 = WG_T * tm, n0 = WG_T * tn;
  const int r0 = s * rows_per_slice;
  const int r1 = r0 + rows_per_slice < rows ? r0 + rows_per_slice : rows;
  const int m_rem = M - (m0 + 64 * wm), n_rem = N - (n0 + 64 * wn);
  const int mb_n = m_rem <= 0 ? 0 : (m_rem > 32 ? 2 : 1), nb_n = n_rem <= 0 ? 0 : (n_rem > 32 ? 2 : 1);
  const bool bias = bpart != nullptr && tn == 0;
  const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(gy), 0, rows * M * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rx =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), 0, ((rows - 1) * ldx + N) * 4, 0x00020000);
  const int col = t & 127, g = t >> 7;
  const int bg = m0 + col < M ? ((r0 + 8 * g) * M + m0 + col) * 4 : WS_OOB;
  const int bx = n0 + col < N ? ((r0 + 8 * g) * ldx + n0 + col) * 4 : WS_OOB;
  const int rgb = M * 4, rxb = ldx * 4;
  f16v acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.0f;
  float bsum = 0.0f;
  const int nch = (r1 - r0 + WS_KC - 1) / WS_KC;
  f8v vg[2], vx[2];  // register slot j & 1 holds chunk j from its load (two iterations before it is staged)
  auto load = [&](int slot, int c) {
    ws_load(rg, bg, rgb, c * WS_KC, vg[slot]);
    ws_load(rx, bx, rxb, c * WS_KC, vx[slot]);
  };
  auto stage = [&](int buf, int slot) {
    ws_split_store(IMG[buf][0], col, g, vg[slot]);
    ws_split_store(IMG[buf][1], col, g, vx[slot]);
  };
  auto frags = [&](int buf, WsFrags& f) {
#pragma unroll
    for (int b = 0; b < 2; ++b) ws_frag(IMG[buf][1], 64 * wn + 32 * b, lane, f.b[b]);
#pragma unroll
    for (int a = 0; a < 2; ++a) ws_frag(IMG[buf][0], 64 * wm + 32 * a, lane, f.a[a]);
  };
  // the bias: this thread's 8 gy rows of the chunk in order (rows past the slice or the matrix are 0 or not staged)
  auto bias_add = [&](int slot, int c) {
    if (c < nch) {
#pragma unroll
      for (int i = 0; i < 8; ++i) bsum += vg[slot][i];
    }
  };
  load(0, 0);
  load(1, 1);
  bias_add(0, 0);
  stage(0, 0);
  load(0, 2);
  __syncthreads();
  WsFrags f0, f1;
  frags(0, f0);
  auto iter = [&](int c, int slot, WsFrags& fc, WsFrags& fn) {
    const int nxt = (c + 1) & 1;
    __builtin_amdgcn_sched_barrier(0);
    bias_add(slot, c + 1);
    stage(nxt, slot);
    load(slot, c + 3);
    acc[0][0] = mfma_bf3f(fc.a[0], fc.b[0], acc[0][0]);
    acc[0][1] = mfma_bf3f(fc.a[0], fc.b[1], acc[0][1]);
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
      __builtin_amdgcn_sched_group_barrier(0x002, 8, 1);
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 1);
      __builtin_amdgcn_sched_group_barrier(0x020, 2, 1);
    }
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
    frags(nxt, fn);
    acc[1][0] = mfma_bf3f(fc.a[1], fc.b[0], acc[1][0]);
    acc[1][1] = mfma_bf3f(fc.a[1], fc.b[1], acc[1][1]);
    __builtin_amdgcn_sched_group_barrier(0x100, 12, 2);
    __builtin_amdgcn_sched_group_barrier(0x008, 12, 2);
  };
  int c = 0;
  for (; c + 1 < nch; c += 2) {
    iter(c, 1, f0, f1);
    iter(c + 1, 0, f1, f0);
  }
  if (c < nch) iter(c, 1, f0, f1);
  __builtin_amdgcn_sched_barrier(0);
  float* P = part + (size_t)s * M * N;
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    if (a >= mb_n) break;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      if (b >= nb_n) break;
      const int n = n0 + 64 * wn + 32 * b + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + 64 * wm + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m < M && n < N) P[(size_t)m * N + n] = acc[a][b][r];
      }
    }
  }
  if (bias) {  // the two row halves of column m, in a fixed order
    __syncthreads();
    float* red = reinterpret_cast<float*>(&IMG[0][0][0]);
    if (g == 1) red[col] = bsum;
    __syncthreads();
    if (g == 0 && m0 + col < M) bpart[(size_t)s * M + m0 + col] = bsum + red[col];
  }
}

// gW[i] = sum_s part[s][i] (i < M N) and gb[m] = sum_s bpart[s][m]: G slice groups per output (thread (g, o) sums
// slices g, g + G, ... in order, eight loads in flight), then the G group sums in order -- a fixed tree for a given
// slice count, so the result is deterministic
__global__ __launch_bounds__(256) void k_wgrad_reduce(const float* __restrict__ part, const float* __restrict__ bpart,
                                                      int slices, int groups, int mn, int m, float* __restrict__ gw,
                                                      float* __restrict__ gb, int accumulate) {
  __shared__ float red[256];
  const int per = 256 / groups, g = threadIdx.x / per, o = threadIdx.x % per;
  const int e = blockIdx.x * per + o;
  const int total = mn + (gb ? m : 0);
  float acc = 0.0f;
  if (e < total) {
    const bool w = e < mn;
    const float* src = w ? part + e : bpart + (e - mn);
    const size_t stride = w ? (size_t)mn : (size_t)m;
    int k = g;
    for (; k + 7 * groups < slices; k += 8 * groups) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = src[(size_t)(k + u * groups) * stride];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; k < slices; k += groups) acc += src[(size_t)k * stride];
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (g == 0 && e < total) {
    float sum = red[o];
    for (int q = 1; q < groups; ++q) sum += red[q * per + o];
    float* dst = e < mn ? gw + e : gb + (e - mn);
    *dst = accumulate ? *dst + sum : sum;  // accumulate: into an existing gradient, as autograd's += would
  }
}

// workgroups per CU the slicing aims at (T1_WGRAD_WG_PER_CU, 1-4: A/B; fewer means fewer, longer slices and
// less partial traffic)
int wg_per_cu() {
  static const int v = [] {
    const char* e = getenv("T1_WGRAD_WG_PER_CU");
    const int k = e ? atoi(e) : 2;
    return k >= 1 && k <= 4 ? k : 2;
  }();
  return v;
}

// T1_WGRAD_STAGED (A/B): 1 (default) k_linear_wgrad_f32s, 0 the first fp32 form k_linear_wgrad_f32
bool wgrad_staged() {
  static const bool v = [] {
    const char* e = getenv("T1_WGRAD_STAGED");
    return !(e && e[0] == '0');
  }();
  return v;
}

struct WgPlan {
  int tiles_m, tiles, slices, rows_per_slice;
};

WgPlan wg_plan(int rows, int M, int N, int cus) {
  WgPlan p;
  p.tiles_m = (M + WG_T - 1) / WG_T;
  p.tiles = p.tiles_m * ((N + WG_T - 1) / WG_T);
  // about wg_per_cu() workgroups per CU, slices of at least WG_MIN_ROWS rows, a multiple of the chunk
  const int want = (wg_per_cu() * cus + p.tiles - 1) / p.tiles;
  const int most = (rows + WG_MIN_ROWS - 1) / WG_MIN_ROWS;
  int sl = want < most ? want : most;
  if (sl < 1) sl = 1;
  int rps = (rows + sl - 1) / sl;
  rps = (rps + WG_ROWS - 1) / WG_ROWS * WG_ROWS;
  p.rows_per_slice = rps;
  p.slices = (rows + rps - 1) / rps;
  return p;
}

int wg_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    return -1;
  return cus;
}

}  // namespace

extern "C" {

long long t1policy_linear_wgrad_workspace_bytes(int rows, int M, int N) {
  if (rows <= 0 || M <= 0 || N <= 0) return -1;
  const int cus = wg_cus();
  if (cus <= 0) return -2;
  const WgPlan p = wg_plan(rows, M, N, cus);
  return (long long)p.slices * ((long long)M * N + M) * 4;
}

int t1policy_linear_wgrad_bf16(const void* gy, const void* x, int rows, int M, int N, void* workspace,
                               long long workspace_bytes, float* grad_weight, float* grad_bias, int accumulate,
                               void* stream) {
  if (!gy || !x || !workspace || !grad_weight || rows <= 0 || M <= 0 || N <= 0) return -1;
  if ((reinterpret_cast<uintptr_t>(gy) & 3u) != 0 || (reinterpret_cast<uintptr_t>(x) & 3u) != 0 ||
      (reinterpret_cast<uintptr_t>(workspace) & 15u) != 0)
    return -1;
  if ((long long)M * N >= (1LL << 31) - M) return -1;
  const int cus = wg_cus();
  if (cus <= 0) return -2;
  const WgPlan p = wg_plan(rows, M, N, cus);
  if (workspace_bytes < (long long)p.slices * ((long long)M * N + M) * 4) return -1;
  float* part = reinterpret_cast<float*>(workspace);
  float* bpart = grad_bias ? part + (size_t)p.slices * M * N : nullptr;
  const dim3 grid(p.tiles, p.slices);
  const uint16_t* g16 = reinterpret_cast<const uint16_t*>(gy);
  const uint16_t* x16 = reinterpret_cast<const uint16_t*>(x);
  const bool gp = (M & 1) == 0, xp = (N & 1) == 0;
  hipStream_t st = (hipStream_t)stream;
  if (gp && xp)
    hipLaunchKernelGGL((k_linear_wgrad_bf16<true, true>), grid, dim3(256), 0, st, g16, x16, rows, M, N, p.tiles_m,
                       p.rows_per_slice, part, bpart);
  else if (gp)
    hipLaunchKernelGGL((k_linear_wgrad_bf16<true, false>), grid, dim3(256), 0, st, g16, x16, rows, M, N, p.tiles_m,
                       p.rows_per_slice, part, bpart);
  else if (xp)
    hipLaunchKernelGGL((k_linear_wgrad_bf16<false, true>), grid, dim3(256), 0, st, g16, x16, rows, M, N, p.tiles_m,
                       p.rows_per_slice, part, bpart);
  else
    hipLaunchKernelGGL((k_linear_wgrad_bf16<false, false>), grid, dim3(256), 0, st, g16, x16, rows, M, N, p.tiles_m,
                       p.rows_per_slice, part, bpart);
  const int total = M * N + (grad_bias ? M : 0);
  const int groups = p.slices <= 8 ? 1 : (p.slices <= 64 ? 4 : 16), per = 256 / groups;
  hipLaunchKernelGGL(k_wgrad_reduce, dim3((total + per - 1) / per), dim3(256), 0, st, part, bpart, p.slices, groups,
                     M * N, M, grad_weight, grad_bias, accumulate);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int t1policy_linear_wgrad_f32x(const float* gy, const float* x, int ldx, int rows, int M, int N, void* workspace,
                               long long workspace_bytes, float* grad_weight, float* grad_bias, int accumulate,
                               void* stream) {
  if (!gy || !x || !workspace || !grad_weight || rows <= 0 || M <= 0 || N <= 0 || ldx < N) return -1;
  if ((reinterpret_cast<uintptr_t>(workspace) & 15u) != 0) return -1;
  if ((long long)M * N >= (1LL << 31) - M || (long long)rows * (M > ldx ? M : ldx) >= (1LL << 31)) return -1;
  const int cus = wg_cus();
  if (cus <= 0) return -2;
  const WgPlan p = wg_plan(rows, M, N, cus);
  if (workspace_bytes < (long long)p.slices * ((long long)M * N + M) * 4) return -1;
  float* part = reinterpret_cast<float*>(workspace);
  float* bpart = grad_bias ? part + (size_t)p.slices * M * N : nullptr;
  hipStream_t st = (hipStream_t)stream;
  if (wgrad_staged() && (long long)rows * M * 4 < WS_OOB && (long long)rows * ldx * 4 < WS_OOB) {
    const int units = p.tiles * p.slices, per_xcd = (units + 7) / 8;
    hipLaunchKernelGGL(k_linear_wgrad_f32s, dim3(8 * per_xcd), dim3(256), 0, st, gy, x, ldx, rows, M, N, p.tiles_m,
                       p.tiles, p.rows_per_slice, units, per_xcd, part, bpart);
  } else if (ldx == N) {
    hipLaunchKernelGGL(k_linear_wgrad_f32, dim3(p.tiles, p.slices), dim3(256), 0, st, gy, x, rows, M, N, p.tiles_m,
                       p.rows_per_slice, part, bpart);
  } else {
    return -1;  // a strided x needs the staged kernel
  }
  const int total = M * N + (grad_bias ? M : 0);
  const int groups = p.slices <= 8 ? 1 : (p.slices <= 64 ? 4 : 16), per = 256 / groups;
  hipLaunchKernelGGL(k_wgrad_reduce, dim3((total + per - 1) / per), dim3(256), 0, st, part, bpart, p.slices, groups,
                     M * N, M, grad_weight, grad_bias, accumulate);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int t1policy_linear_wgrad_f32(const float* gy, const float* x, int rows, int M, int N, void* workspace,
                              long long workspace_bytes, float* grad_weight, float* grad_bias, int accumulate,
                              void* stream) {
  return t1policy_linear_wgrad_f32x(gy, x, N, rows, M, N, workspace, workspace_bytes, grad_weight, grad_bias,
                                    accumulate, stream);
}

}  // extern "C"
