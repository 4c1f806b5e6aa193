// Probe: a 16-byte global load / non-temporal load from a 4-byte-aligned (not 16-byte-aligned) address -- whether the
// MI355X returns the four floats at that address (the history shift's source window, k_dyn6).  Prints PASS / FAIL.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void k_probe16(const unsigned short* in, unsigned short* out, int n) {  // 2-byte aligned 16-B loads
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  const u4 v = *reinterpret_cast<const u4*>(in + 8 * t + 3);
  const unsigned w[4] = {v.x, v.y, v.z, v.w};
  for (int k = 0; k < 4; ++k) { out[8 * t + 2 * k] = (unsigned short)(w[k] & 0xffffu); out[8 * t + 2 * k + 1] = (unsigned short)(w[k] >> 16); }
}
__global__ void k_probe(const float* in, float* out, int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const float* src = in + 4 * t + 3;  // 12 bytes past a 16-byte boundary
  const f4 v = __builtin_nontemporal_load(reinterpret_cast<const f4*>(src));
  const f4 w = *reinterpret_cast<const f4*>(in + 4 * t + 1);
  out[8 * t + 0] = v.x; out[8 * t + 1] = v.y; out[8 * t + 2] = v.z; out[8 * t + 3] = v.w;
  out[8 * t + 4] = w.x; out[8 * t + 5] = w.y; out[8 * t + 6] = w.z; out[8 * t + 7] = w.w;
}

int main() {
  const int n = 4096;
  std::vector<float> h(4 * n + 16);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)i;
  float *din, *dout;
  if (hipMalloc(&din, h.size() * 4) != hipSuccess || hipMalloc(&dout, 8 * n * 4) != hipSuccess) return 2;
  (void)hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_probe, dim3(n / 256), dim3(256), 0, 0, din, dout, n);
  const hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) { printf("FAIL launch: %s\n", hipGetErrorString(e)); return 1; }
  std::vector<float> o(8 * n);
  (void)hipMemcpy(o.data(), dout, 8 * n * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int t = 0; t < n; ++t)
    for (int k = 0; k < 4; ++k) {
      bad += o[8 * t + k] != (float)(4 * t + 3 + k);
      bad += o[8 * t + 4 + k] != (float)(4 * t + 1 + k);
    }
  printf("%s (4-byte aligned): %d wrong of %d\n", bad ? "FAIL" : "PASS", bad, 8 * n);
  std::vector<unsigned short> h16(8 * n + 16);
  for (size_t i = 0; i < h16.size(); ++i) h16[i] = (unsigned short)(i & 0xffff);
  unsigned short *i16, *o16;
  if (hipMalloc(&i16, h16.size() * 2) != hipSuccess || hipMalloc(&o16, 8 * n * 2) != hipSuccess) return 2;
  (void)hipMemcpy(i16, h16.data(), h16.size() * 2, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_probe16, dim3(n / 256), dim3(256), 0, 0, i16, o16, n);
  const hipError_t e2 = hipDeviceSynchronize();
  if (e2 != hipSuccess) { printf("FAIL launch (2-byte): %s\n", hipGetErrorString(e2)); return 1; }
  std::vector<unsigned short> r16(8 * n);
  (void)hipMemcpy(r16.data(), o16, 8 * n * 2, hipMemcpyDeviceToHost);
  int bad2 = 0;
  for (int t = 0; t < n; ++t)
    for (int k = 0; k < 8; ++k) bad2 += r16[8 * t + k] != (unsigned short)((8 * t + 3 + k) & 0xffff);
  printf("%s (2-byte aligned): %d wrong of %d\n", bad2 ? "FAIL" : "PASS", bad2, 8 * n);
  return (bad || bad2) ? 1 : 0;
}
