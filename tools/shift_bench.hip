// Microbenchmark of the history shift (t1env_device.h shift_history) at the config-5 size: variants of the
// load shape, grid and cache policy against a plain float4 copy of the same bytes (the achievable HBM rate).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/shift_bench tools/shift_bench.hip && /tmp/shift_bench [num_envs]
// Prints one line per variant: average kernel time (HIP events, 50 launches) and algorithmic GB/s
// (read + write of the shifted older frames), and checks every variant's output against the current kernel.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../ti5_isaacgym_amd/csrc/t1env_device.h"

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

using namespace t1;

__global__ __launch_bounds__(256) void k_cur(ShiftArgs S) {
  shift_history(S, (int64_t)blockIdx.x * blockDim.x + threadIdx.x, (int64_t)gridDim.x * blockDim.x);
}

// unaligned 16-B source loads (dword-aligned; gfx9 global loads take them), aligned 16-B stores
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
typedef float f4a __attribute__((ext_vector_type(4)));

template <int F, int H, int U, bool NT>
__device__ __forceinline__ void shift_unal(const float* __restrict__ in, float* __restrict__ out, int64_t total,
                                           int64_t t0, int64_t stride) {
  constexpr int ROW = F * H;
  const int64_t n4 = (total + 3) / 4;
  for (int64_t base = t0; base < n4; base += U * stride) {
    f4a v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      int64_t s = (base + u * stride) * 4 + F;
      if (s + 4 > total) s = total - 4;  // clamp (tail handled below)
      const f4u* p = reinterpret_cast<const f4u*>(in + s);
      if constexpr (NT) v[u] = __builtin_nontemporal_load(p);
      else v[u] = *p;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i4 = base + u * stride;
      if (i4 >= n4) break;
      const int64_t i = i4 * 4;
      const int64_t row = i / ROW;
      const int col = (int)(i - row * ROW);
      if (col + 3 < ROW - F && i + F + 4 <= total) {
        f4a* q = reinterpret_cast<f4a*>(out + i);
        if constexpr (NT) __builtin_nontemporal_store(v[u], q);
        else *q = v[u];
      } else {
        for (int k = 0; k < 4; ++k) {
          const int64_t e = i + k;
          if (e >= total) break;
          const int64_t r = e / ROW;
          if ((int)(e - r * ROW) < ROW - F) out[e] = in[e + F];
        }
      }
    }
  }
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_unal(ShiftArgs S) {
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, st = (int64_t)gridDim.x * blockDim.x;
  shift_unal<T1_NOBS, T1_HIST, U, NT>(S.obs_in, S.obs_out, S.total_obs, t0, st);
  shift_unal<T1_NPRIV, T1_CHIST, U, NT>(S.priv_in, S.priv_out, S.total_priv, t0, st);
}

// row-blocked: one workgroup per `rows` consecutive rows (contiguous span), no grid stride
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_rows(ShiftArgs S, int rows) {
  const int64_t r0 = (int64_t)blockIdx.x * rows;
  constexpr int64_t RO = T1_NOBS * T1_HIST, RP = T1_NPRIV * T1_CHIST;
  // treat the rows' span as a sub-buffer: the flat shift never crosses a row for stored columns
  const int64_t nrow = S.total_obs / RO;
  int64_t r1 = r0 + rows;
  if (r1 > nrow) r1 = nrow;
  if (r0 >= r1) return;
  shift_unal<T1_NOBS, T1_HIST, U, NT>(S.obs_in + r0 * RO, S.obs_out + r0 * RO, (r1 - r0) * RO, threadIdx.x, 256);
  shift_unal<T1_NPRIV, T1_CHIST, U, NT>(S.priv_in + r0 * RP, S.priv_out + r0 * RP, (r1 - r0) * RP, threadIdx.x,
                                         256);
}

// ceiling: aligned float4 copy of the same number of bytes
__global__ __launch_bounds__(256) void k_copy(const float4* __restrict__ in, float4* __restrict__ out, int64_t n4) {
  const int64_t st = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += 4 * st) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = i + u * st < n4 ? in[i + u * st] : make_float4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + u * st < n4) out[i + u * st] = v[u];
  }
}

int main(int argc, char** argv) {
  const int64_t N = argc > 1 ? atoll(argv[1]) : 32768;
  const int64_t to = N * T1_NOBS * T1_HIST, tp = N * T1_NPRIV * T1_CHIST;
  const double alg = 2.0 * 4.0 * (double)N * (T1_NOBS * (T1_HIST - 1) + T1_NPRIV * (T1_CHIST - 1));
  float *oi, *oo, *pi, *po, *ref_o, *ref_p;
  CK(hipMalloc(&oi, to * 4));
  CK(hipMalloc(&oo, to * 4));
  CK(hipMalloc(&pi, tp * 4));
  CK(hipMalloc(&po, tp * 4));
  CK(hipMalloc(&ref_o, to * 4));
  CK(hipMalloc(&ref_p, tp * 4));
  {
    std::vector<float> h(to);
    for (int64_t i = 0; i < to; ++i) h[i] = (float)(i % 100003) * 0.5f;
    CK(hipMemcpy(oi, h.data(), to * 4, hipMemcpyHostToDevice));
    std::vector<float> g(tp);
    for (int64_t i = 0; i < tp; ++i) g[i] = (float)(i % 7919) * 0.25f;
    CK(hipMemcpy(pi, g.data(), tp * 4, hipMemcpyHostToDevice));
  }
  ShiftArgs S{oi, ref_o, pi, ref_p, to, tp};
  CK(hipMemset(ref_o, 0, to * 4));
  CK(hipMemset(ref_p, 0, tp * 4));
  hipLaunchKernelGGL(k_cur, dim3(1024), dim3(256), 0, 0, S);
  CK(hipDeviceSynchronize());
  std::vector<float> ro(to), rp(tp), xo(to), xp(tp);
  CK(hipMemcpy(ro.data(), ref_o, to * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(rp.data(), ref_p, tp * 4, hipMemcpyDeviceToHost));
  ShiftArgs T{oi, oo, pi, po, to, tp};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch, bool check, double bytes = 0.0) {
    if (bytes == 0.0) bytes = alg;
    CK(hipMemset(oo, 0, to * 4));
    CK(hipMemset(po, 0, tp * 4));
    launch();
    CK(hipDeviceSynchronize());
    bool ok = true;
    if (check) {
      CK(hipMemcpy(xo.data(), oo, to * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(xp.data(), po, tp * 4, hipMemcpyDeviceToHost));
      for (int64_t i = 0; i < to && ok; ++i) ok = xo[i] == ro[i];
      for (int64_t i = 0; i < tp && ok; ++i) ok = xp[i] == rp[i];
    }
    for (int w = 0; w < 5; ++w) launch();
    CK(hipEventRecord(e0, 0));
    const int reps = 50;
    for (int w = 0; w < reps; ++w) launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("%-28s %8.4f ms  %7.1f GB/s  %s\n", name, ms, bytes / (ms * 1e-3) / 1e9, check ? (ok ? "ok" : "MISMATCH") : "-");
    fflush(stdout);
  };
  // the obs buffers only (both are to floats; to is a multiple of 4): read + write of 2 x 4 x to bytes
  const int64_t n4 = to / 4;
  for (int g : {1024, 4096})
    run((std::string("copy g") + std::to_string(g)).c_str(),
        [&] { hipLaunchKernelGGL(k_copy, dim3(g), dim3(256), 0, 0, (const float4*)oi, (float4*)oo, n4); }, false,
        8.0 * (double)to);
  for (int g : {512, 1024, 2048, 4096})
    run((std::string("cur g") + std::to_string(g)).c_str(),
        [&] { hipLaunchKernelGGL(k_cur, dim3(g), dim3(256), 0, 0, T); }, true);
  for (int g : {1024, 2048, 4096}) {
    run((std::string("unal4 g") + std::to_string(g)).c_str(),
        [&] { hipLaunchKernelGGL((k_unal<4, false>), dim3(g), dim3(256), 0, 0, T); }, true);
    run((std::string("unal4 nt g") + std::to_string(g)).c_str(),
        [&] { hipLaunchKernelGGL((k_unal<4, true>), dim3(g), dim3(256), 0, 0, T); }, true);
    run((std::string("unal8 g") + std::to_string(g)).c_str(),
        [&] { hipLaunchKernelGGL((k_unal<8, false>), dim3(g), dim3(256), 0, 0, T); }, true);
  }
  for (int rows : {4, 8, 16}) {
    const int g = (int)((N + rows - 1) / rows);
    run((std::string("rows") + std::to_string(rows)).c_str(),
        [&] { hipLaunchKernelGGL((k_rows<4, false>), dim3(g), dim3(256), 0, 0, T, rows); }, true);
    run((std::string("rows nt") + std::to_string(rows)).c_str(),
        [&] { hipLaunchKernelGGL((k_rows<4, true>), dim3(g), dim3(256), 0, 0, T, rows); }, true);
  }
  return 0;
}
