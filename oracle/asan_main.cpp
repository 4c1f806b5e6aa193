// asan_main.cpp -- TEST INFRASTRUCTURE: host build of the product dynamics header (oracle/dyn_cpu.cpp) under
// AddressSanitizer + UndefinedBehaviorSanitizer (tests/test_dynamics.py::test_host_dynamics_under_sanitizers).
// Reads a t1env_model blob (written by the test from the URDF-derived model) and runs both substep compositions
// (assembled / k_dyn4 split) in fp32 and fp64 on random states over a rough height field, with contact.
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#include "dyn_cpu.cpp"

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  t1env_model model;
  FILE* f = fopen(argv[1], "rb");
  if (!f || fread(&model, sizeof(model), 1, f) != 1) return 3;
  fclose(f);
  const int N = 16, rows = 40, cols = 40;
  std::vector<int16_t> hf(rows * cols);
  unsigned s = 12345u;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (float)((s >> 8) & 0xffff) / 65536.0f; };
  for (auto& h : hf) h = (int16_t)(rnd() * 40.0f - 20.0f);
  for (int flags = 0; flags < 4; ++flags) {
    std::vector<float> root(N * 13, 0.0f), dof(N * 24, 0.0f), tau(N * 12), bm(N), ls(N * 12, 1.0f), cd(N * 3, 0.0f),
        arm(N * 12, 0.1f), fr(N, 0.8f), rst(N, 0.3f), vimp(N * 6, 0.0f), rigid(N * 169), contact(N * 39), ext(N * 3, 0.0f);
    const float q0[6] = {0.0f, 0.0f, -0.3f, 0.6f, -0.3f, 0.0f};
    for (int n = 0; n < N; ++n) {
      root[n * 13 + 0] = 1.5f + rnd();
      root[n * 13 + 1] = 1.5f + rnd();
      root[n * 13 + 2] = 0.90f + 0.06f * rnd();
      root[n * 13 + 6] = 1.0f;
      for (int i = 7; i < 13; ++i) root[n * 13 + i] = 0.6f * rnd() - 0.3f;
      for (int j = 0; j < 12; ++j) {
        dof[n * 24 + 2 * j] = q0[j % 6] + 0.6f * rnd() - 0.3f;
        dof[n * 24 + 2 * j + 1] = 4.0f * rnd() - 2.0f;
        tau[n * 12 + j] = 60.0f * rnd() - 30.0f;
      }
      bm[n] = model.mass[0];
      ext[n * 3 + 0] = 100.0f * rnd();
    }
    const int rc = t1dyn_substeps(&model, N, flags, root.data(), dof.data(), tau.data(), bm.data(), ls.data(), cd.data(),
                                  arm.data(), fr.data(), rst.data(), vimp.data(), ext.data(), 0.001f, 20, hf.data(), rows, cols, 0.1f, 0.005f,
                                  1.0f, 2, rigid.data(), contact.data());
    if (rc) return 4;
    for (float v : root)
      if (!(v == v)) return 5;  // NaN
  }
  printf("ok\n");
  return 0;
}
