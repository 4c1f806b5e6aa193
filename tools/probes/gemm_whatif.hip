// Dev probe: what bounds k_gemm_nt_f32x3 (csrc/t1policy_gemm.hip)?  Built once per T1_GEMM_WHATIF value (timing-only
// what-if builds: bit 0 no in-loop global loads, 1 no LDS stores, 2 one MFMA per product, 3 no split); times the
// update's two largest forward shapes and one dgrad shape with HIP events.  Results are wrong by construction in the
// what-if builds; only the time is read.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -DT1_GEMM_WHATIF=<bits> -o gemm_whatif_<bits> tools/probes/gemm_whatif.hip
#include "../../ti5_isaacgym_amd/csrc/t1policy_gemm.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

int main() {
  struct Shape { int R, N, K; };
  const Shape shapes[] = {{49152, 256, 512}, {49152, 302, 512}, {49152, 256, 768}, {49152, 768, 219}};
  size_t maxa = 0, maxb = 0, maxc = 0;
  for (const Shape& s : shapes) {
    maxa = std::max(maxa, (size_t)s.R * s.K);
    maxb = std::max(maxb, (size_t)s.N * s.K);
    maxc = std::max(maxc, (size_t)s.R * s.N);
  }
  float *A, *B, *C;
  if (hipMalloc(&A, maxa * 4) || hipMalloc(&B, maxb * 4) || hipMalloc(&C, maxc * 4)) return 1;
  std::vector<float> h(maxa);
  for (size_t i = 0; i < maxa; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.0f - 0.5f;
  hipMemcpy(A, h.data(), maxa * 4, hipMemcpyHostToDevice);
  hipMemcpy(B, h.data(), maxb * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  printf("{\"whatif\": %d, \"shapes\": [", T1_GEMM_WHATIF);
  const char* only = getenv("GEMM_SHAPE");  // one shape only (counter passes)
  for (int i = 0; i < 4; ++i) {
    if (only && atoi(only) != i) continue;
    const Shape s = shapes[i];
    for (int w = 0; w < 5; ++w) t1policy_gemm_nt_f32(A, B, nullptr, nullptr, C, s.R, s.N, s.K, 0, nullptr);
    hipEventRecord(e0, nullptr);
    const int reps = 50;
    for (int r = 0; r < reps; ++r) t1policy_gemm_nt_f32(A, B, nullptr, nullptr, C, s.R, s.N, s.K, 0, nullptr);
    hipEventRecord(e1, nullptr);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / reps, tf = 2.0 * s.R * s.N * s.K / (us * 1e-6) / 1e12;
    printf("%s{\"R\": %d, \"N\": %d, \"K\": %d, \"us\": %.2f, \"tflops\": %.1f}", i ? ", " : "", s.R, s.N, s.K, us, tf);
  }
  printf("]}\n");
  return hipDeviceSynchronize() == hipSuccess ? 0 : 2;
}
