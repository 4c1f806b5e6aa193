// pk_issue_bench.hip -- issue cost of packed vs scalar fp32 VALU for ONE wave alone on its SIMD (the k_dyn4
// leg wave's situation: 363 VGPRs, one wave per SIMD).  Each variant times a fully unrolled block of
// instructions with s_memtime (shader clock) on a single wave; cycles per instruction are printed.
//   hipcc --offload-arch=gfx950 -O3 -o tools/pk_issue_bench tools/pk_issue_bench.hip && ./tools/pk_issue_bench
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

constexpr int REP = 64;  // repetitions of the unrolled body

#define FMA1(a) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a) : "v"(x), "v"(y))
#define PKFMA1(a) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(a) : "v"(px), "v"(py))
#define PKMUL1(a) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(a) : "v"(px))
#define PKADD1(a) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a) : "v"(px))
#define MUL1(a) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a) : "v"(x))

// variant: 0 scalar fma x8 independent, 1 pk_fma x8 independent, 2 scalar fma dependent, 3 pk_fma dependent,
// 4 pk_mul x8 indep, 5 pk_add x8 indep, 6 scalar mul x8 indep, 7 scalar fma x4 indep, 8 pk_fma x4 indep
__global__ void k_bench(int variant, float seed, unsigned long long* cyc, float* sink) {
  float x = seed + threadIdx.x, y = seed * 0.5f;
  f2 px = {x, y}, py = {y, x};
  float a0 = x, a1 = y, a2 = x + 1, a3 = y + 1, a4 = x + 2, a5 = y + 2, a6 = x + 3, a7 = y + 3;
  f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}, p4 = {a1, a0}, p5 = {a3, a2}, p6 = {a5, a4},
     p7 = {a7, a6};
  unsigned long long t0 = stamp();
  switch (variant) {
    case 0:
      _Pragma("unroll") for (int r = 0; r < REP; ++r) { FMA1(a0); FMA1(a1); FMA1(a2); FMA1(a3); FMA1(a4); FMA1(a5); FMA1(a6); FMA1(a7); }
      break;
    case 1:
      _Pragma("unroll") for (int r = 0; r < REP; ++r) { PKFMA1(p0); PKFMA1(p1); PKFMA1(p2); PKFMA1(p3); PKFMA1(p4); PKFMA1(p5); PKFMA1(p6); PKFMA1(p7); }
      break;
    case 2:
      _Pragma("unroll") for (int r = 0; r < 8 * REP; ++r) FMA1(a0);
      break;
    case 3:
      _Pragma("unroll") for (int r = 0; r < 8 * REP; ++r) PKFMA1(p0);
      break;
    case 4:
      _Pragma("unroll") for (int r = 0; r < REP; ++r) { PKMUL1(p0); PKMUL1(p1); PKMUL1(p2); PKMUL1(p3); PKMUL1(p4); PKMUL1(p5); PKMUL1(p6); PKMUL1(p7); }
      break;
    case 5:
      _Pragma("unroll") for (int r = 0; r < REP; ++r) { PKADD1(p0); PKADD1(p1); PKADD1(p2); PKADD1(p3); PKADD1(p4); PKADD1(p5); PKADD1(p6); PKADD1(p7); }
      break;
    case 6:
      _Pragma("unroll") for (int r = 0; r < REP; ++r) { MUL1(a0); MUL1(a1); MUL1(a2); MUL1(a3); MUL1(a4); MUL1(a5); MUL1(a6); MUL1(a7); }
      break;
    case 7:
      _Pragma("unroll") for (int r = 0; r < 2 * REP; ++r) { FMA1(a0); FMA1(a1); FMA1(a2); FMA1(a3); }
      break;
    case 8:
      _Pragma("unroll") for (int r = 0; r < 2 * REP; ++r) { PKFMA1(p0); PKFMA1(p1); PKFMA1(p2); PKFMA1(p3); }
      break;
  }
  unsigned long long t1 = stamp();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  f2 ps = p0 + p1 + p2 + p3 + p4 + p5 + p6 + p7;
  sink[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + ps.x + ps.y;
}

// wall-clock calibration: ITER x 64 instructions per wave, timed with HIP events.  grid 1: one wave alone;
// grid 1024 x 64: one wave on every SIMD (256 CUs x 4), the k_dyn4 situation at full occupancy of one wave/SIMD
constexpr int ITER = 20000;
__global__ __launch_bounds__(64) void k_wall(int variant, float seed, float* sink) {
  float x = seed + threadIdx.x, y = seed * 0.5f;
  f2 px = {x, y}, py = {y, x};
  float a0 = x, a1 = y, a2 = x + 1, a3 = y + 1, a4 = x + 2, a5 = y + 2, a6 = x + 3, a7 = y + 3;
  f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}, p4 = {a1, a0}, p5 = {a3, a2}, p6 = {a5, a4},
     p7 = {a7, a6};
  for (int it = 0; it < ITER; ++it) {
    if (variant == 0) {
      _Pragma("unroll") for (int r = 0; r < 8; ++r) { FMA1(a0); FMA1(a1); FMA1(a2); FMA1(a3); FMA1(a4); FMA1(a5); FMA1(a6); FMA1(a7); }
    } else if (variant == 1) {
      _Pragma("unroll") for (int r = 0; r < 8; ++r) { PKFMA1(p0); PKFMA1(p1); PKFMA1(p2); PKFMA1(p3); PKFMA1(p4); PKFMA1(p5); PKFMA1(p6); PKFMA1(p7); }
    } else if (variant == 2) {
      _Pragma("unroll") for (int r = 0; r < 64; ++r) FMA1(a0);
    } else {
      _Pragma("unroll") for (int r = 0; r < 64; ++r) PKFMA1(p0);
    }
  }
  f2 ps = p0 + p1 + p2 + p3 + p4 + p5 + p6 + p7;
  sink[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + ps.x + ps.y;
}

int main() {
  const char* names[] = {"v_fma_f32 x8 indep",   "v_pk_fma_f32 x8 indep", "v_fma_f32 dependent", "v_pk_fma_f32 dependent",
                         "v_pk_mul_f32 x8 indep", "v_pk_add_f32 x8 indep", "v_mul_f32 x8 indep",  "v_fma_f32 x4 indep",
                         "v_pk_fma_f32 x4 indep"};
  unsigned long long* cyc;
  float* sink;
  hipMalloc(&cyc, 256 * sizeof(unsigned long long));
  hipMalloc(&sink, 256 * 256 * sizeof(float));
  // one wave alone (grid 1 x 64 threads)
  for (int v = 0; v < 9; ++v) {
    for (int it = 0; it < 3; ++it) hipLaunchKernelGGL(k_bench, dim3(1), dim3(64), 0, 0, v, 1.0f, cyc, sink);
    hipDeviceSynchronize();
    unsigned long long h = 0;
    hipMemcpy(&h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    const int n = 8 * REP;
    printf("%-26s %8llu cycles / %d instr = %6.2f cyc/instr\n", names[v], h, n, (double)h / n);
  }
  const char* wn[] = {"v_fma_f32 x8 indep", "v_pk_fma_f32 x8 indep", "v_fma_f32 dependent", "v_pk_fma_f32 dependent"};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float* sink2;
  hipMalloc(&sink2, 1024 * 64 * sizeof(float));
  int clk_khz = 0;
  hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
  printf("device clock attribute: %d MHz\n", clk_khz / 1000);
  for (int grid : {1, 1024})
    for (int v = 0; v < 4; ++v) {
      hipLaunchKernelGGL(k_wall, dim3(grid), dim3(64), 0, 0, v, 1.0f, sink2);  // warm-up (clock ramp)
      hipEventRecord(e0);
      hipLaunchKernelGGL(k_wall, dim3(grid), dim3(64), 0, 0, v, 1.0f, sink2);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double ns = ms * 1e6 / (64.0 * ITER);
      printf("wall grid %4d  %-24s %7.3f ns/instr = %5.2f cyc/instr at %d MHz\n", grid, wn[v], ns,
             ns * clk_khz / 1e6, clk_khz / 1000);
    }
  hipFree(cyc);
  hipFree(sink);
  hipFree(sink2);
  return 0;
}
