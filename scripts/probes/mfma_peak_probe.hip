// Sustained bf16 MFMA throughput of the whole chip under its power limit (the practical GEMM ceiling).
//
//   hipcc -O3 --offload-arch=gfx950 scripts/probes/mfma_peak_probe.hip -o scripts/probes/mfma_peak_probe
//   ./scripts/probes/mfma_peak_probe [iters]
//
// Every wave issues back-to-back v_mfma_f32_32x32x16_bf16 on four independent accumulators (no memory traffic
// inside the loop), 2 waves per SIMD on every CU, for ~50-100 ms of wall time.  Operands are loaded once from a
// buffer filled with uniform random bf16 values or with zeros: the chip's clock under load (DVFS) depends on the
// data (MI355X_MICROARCH.md, DVFS give-back), so the random-operand number is the ceiling a real bf16 GEMM can
// approach, the zero-operand one what the MFMA pipe does at a higher clock.  Reports TFLOP/s per run; the
// kernel's dependent-register outputs are written back so nothing is dead code.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                                              \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));                    \
      std::exit(1);                                                                           \
    }                                                                                         \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

// the same with v_mfma_f32_16x16x32_bf16 (half the FLOP per instruction at half the cycles): 8 accumulators
__global__ __launch_bounds__(512) void mfma16_loop(const uint4* __restrict__ src, float* __restrict__ out, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint4 a4 = src[(tid * 2) & 4095], b4 = src[(tid * 2 + 1) & 4095];
  const bf16x8 a = __builtin_bit_cast(bf16x8, a4), b = __builtin_bit_cast(bf16x8, b4);
  f32x4 c[8] = {};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < 8; ++q)
        c[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16((q & 1) ? a : b, (q & 2) ? b : a, c[q], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < 8; ++q) s += c[q][0] + c[q][1] + c[q][2] + c[q][3];
  out[tid] = s;
}

// the weight-gradient GEMM's inner loop without memory: 8 x 4 distinct operand fragments, 32 accumulators
// (csrc/gemm_tn.hip step(): acc[i][j] = mfma(b[j], a[i], acc[i][j])) -- register-file operand traffic of a real tile
__global__ __launch_bounds__(512) void mfma16_tile_loop(const uint4* __restrict__ src, float* __restrict__ out,
                                                         int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  bf16x8 a[8], b[4];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = __builtin_bit_cast(bf16x8, src[(tid * 12 + i) & 4095]);
#pragma unroll
  for (int j = 0; j < 4; ++j) b[j] = __builtin_bit_cast(bf16x8, src[(tid * 12 + 8 + j) & 4095]);
  f32x4 c[8][4] = {};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) c[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], c[i][j], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) s += c[i][j][0] + c[i][j][1] + c[i][j][2] + c[i][j][3];
  out[tid] = s;
}

__global__ __launch_bounds__(512) void mfma_loop(const uint4* __restrict__ src, float* __restrict__ out, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint4 a4 = src[(tid * 2) & 4095], b4 = src[(tid * 2 + 1) & 4095];
  const bf16x8 a = __builtin_bit_cast(bf16x8, a4), b = __builtin_bit_cast(bf16x8, b4);
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, a, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, b, c3, 0, 0, 0);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) s += c0[j] + c1[j] + c2[j] + c3[j];
  out[tid] = s;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 20000;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int blocks = cus, threads = 512;               // 8 waves per CU = 2 per SIMD
  std::vector<uint16_t> host(4096 * 8);
  uint32_t x = 12345u;
  for (auto& h : host) {                                // uniform random bf16 in about (-1, 1)
    x = x * 1664525u + 1013904223u;
    const float f = ((x >> 8) * (1.0f / 16777216.0f)) * 2.f - 1.f;
    uint32_t u;
    std::memcpy(&u, &f, 4);
    h = (uint16_t)(u >> 16);
  }
  uint4* d_rand;
  uint4* d_zero;
  float* d_out;
  CHECK(hipMalloc(&d_rand, host.size() * 2));
  CHECK(hipMalloc(&d_zero, host.size() * 2));
  CHECK(hipMalloc(&d_out, (size_t)blocks * threads * 4));
  CHECK(hipMemcpy(d_rand, host.data(), host.size() * 2, hipMemcpyHostToDevice));
  CHECK(hipMemset(d_zero, 0, host.size() * 2));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  // per launch: 16 MFMAs of 32x32x16 per iteration and wave; the 16x16x32 loop issues 32 (same FLOP)
  const double flop = 2.0 * 32 * 32 * 16 * 16.0 * iters * (blocks * threads / 64.0);
  for (int round = 0; round < 3; ++round) {
    for (int z = 0; z < 6; ++z) {
      const uint4* src = (z & 1) ? d_zero : d_rand;
      auto kern = z < 2 ? mfma_loop : z < 4 ? mfma16_loop : mfma16_tile_loop;
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, src, d_out, iters / 4);   // warm
      CHECK(hipEventRecord(e0));
      for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, src, d_out, iters);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms = 0.f;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      std::printf("round %d %s %-6s operands: %8.2f ms for 5 launches, %7.1f TFLOP/s bf16 (%d CUs, %d waves/CU)\n",
                  round, z < 2 ? "32x32x16" : z < 4 ? "16x16x32" : "16x16x32 tile (8x4 frags)", (z & 1) ? "zero" : "random",
                  ms, 5.0 * flop / (ms * 1e-3) / 1e12,
                  cus, threads / 64);
    }
  }
  CHECK(hipGetLastError());
  CHECK(hipFree(d_rand));
  CHECK(hipFree(d_zero));
  CHECK(hipFree(d_out));
  return 0;
}
