// Ablation driver for csrc/gemm_nt.hip: time the NT GEMM on the TinyGPT-A per-layer shapes, built
// with DLTB_NT_ABL = 0 (full), 1 (no MFMA), 2 (no LDS-DMA in the k-loop), 3 (no LDS reads / MFMA).
//   for a in 0 1 2 3; do hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc -DDLTB_NT_ABL=$a \
//       -x hip csrc/gemm_nt.hip -x c++ scripts/probes/gemm_nt_abl.cpp -o gemm_nt_abl$a; done
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "launchers.h"

int main(int argc, char** argv) {
  const int abl = argc > 1 ? atoi(argv[1]) : -1;
  struct P { const char* name; int N, K, cfg; };
  const P ps[] = {{"out.fwd 128x64k64", 1024, 1024, 0}, {"fc2.fwd 128x64k64", 1024, 4096, 0},
                  {"qkv.fwd 128x192k32", 3072, 1024, 2}, {"fc1.fwd 128x256k32", 4096, 1024, 3},
                  {"fc1.fwd 256x128k32", 4096, 1024, 4}, {"fc2.fwd 64x128k64", 1024, 4096, 5}};
  const int M = 2048;
  void *a, *b, *c;
  hipMalloc(&a, (size_t)M * 4096 * 2);
  hipMalloc(&b, (size_t)4096 * 4096 * 2);
  hipMalloc(&c, (size_t)M * 4096 * 2);
  hipMemset(a, 0x3c, (size_t)M * 4096 * 2);
  hipMemset(b, 0x3c, (size_t)4096 * 4096 * 2);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (const P& p : ps) {
    for (int i = 0; i < 5; ++i) dltb_gemm_nt(a, b, c, nullptr, p.K, p.K, p.N, M, p.N, p.K, 0, p.cfg, 4, 0);
    hipDeviceSynchronize();
    const int reps = 50;
    hipEventRecord(e0);
    for (int i = 0; i < reps; ++i) dltb_gemm_nt(a, b, c, nullptr, p.K, p.K, p.N, M, p.N, p.K, 0, p.cfg, 4, 0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / reps;
    printf("abl %d  %-20s %7.2f us  %6.0f TF/s\n", abl, p.name, us, 2.0 * M * p.N * p.K / us / 1e6);
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
