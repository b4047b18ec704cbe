// Per-CU operand-stream probe (gfx950): how fast can one workgroup per CU pull GEMM-shaped tiles
// (rows of 128 B at a row stride) out of an L2-resident buffer, by LDS-DMA versus register loads?
//
//   hipcc --offload-arch=gfx950 -O3 -o l2_stream_probe l2_stream_probe.hip && ./l2_stream_probe
//
// Each workgroup streams `steps` stages; a stage = ROWS rows x 128 B (64 bf16 of K) at byte stride
// `stride`, row panel chosen per workgroup inside a buffer that every XCD's L2 holds after the warm
// pass.  Modes: 0 = LDS-DMA ring (global_load_lds_dwordx4, counted vmcnt, one s_barrier per stage,
// NSTAGE-1 stages in flight; the GEMM's pipeline without the MFMAs); 1 = global_load_dwordx4 into
// registers (DEPTH stages in flight, xor-consumed); 2 = mode 1 + ds_write_b128 of every stage.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

template <int N>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

__device__ __forceinline__ void glds16(const void* gsrc, const void* lds_dst) {
  const uint32_t lds = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)lds_dst);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds)
               : "memory");
}

template <int ROWS, int NSTAGE>
__global__ __launch_bounds__(256, 1) void probe_dma(const char* buf, long stride, long panel, int steps,
                                                   int* sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NI = ROWS * 8 / 256;      // 16-B pieces per lane per stage
  constexpr int STAGE = ROWS * 128;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const char* base = buf + (long)(blockIdx.x % 64) * panel;
  auto load = [&](int s, int slot) {
    const long koff = (long)(s & 15) * 128;     // 16 k-steps then wrap (stays in L2)
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int lin = (w * NI + i) * 64 + lane, row = lin >> 3, ch = lin & 7;
      glds16(base + row * stride + koff + ch * 16, smem + slot * STAGE + (w * NI + i) * 1024);
    }
  };
  for (int s = 0; s < NSTAGE - 1; ++s) load(s, s);
  int slot = 0;
  for (int s = 0; s < steps; ++s) {
    const int ahead = min(steps - 1 - s, NSTAGE - 2);
    if (ahead >= NSTAGE - 2) wait_vm<(NSTAGE - 2) * NI>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    if (s + NSTAGE - 1 < steps) load(s + NSTAGE - 1, slot == 0 ? NSTAGE - 1 : slot - 1);
    slot = slot == NSTAGE - 1 ? 0 : slot + 1;
  }
  wait_vm<0>();
  __syncthreads();
  if (tid == 0) sink[blockIdx.x] = smem[lane];
}

// mode 3 (round 6): the DMA ring issued the way csrc/gemm_tn.hip does it -- wave-uniform base pointer + per-lane 32-bit
// offsets (saddr form), LDS destinations precomputed, two pieces per asm block with m0 saved once
__device__ __forceinline__ void glds16x2(uint64_t sbase, uint32_t v0, uint32_t v1, uint32_t l0, uint32_t l1) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %3\n\t"
               "s_mov_b32 m0, %5\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %3\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(v0), "v"(v1), "s"(sbase), "s"(l0), "s"(l1)
               : "memory");
}

template <int ROWS, int NSTAGE>
__global__ __launch_bounds__(256, 1) void probe_dma_sv(const char* buf, long stride, long panel, int steps,
                                                      int* sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NI = ROWS * 8 / 256;
  static_assert(NI % 2 == 0, "pieces come in pairs");
  constexpr int STAGE = ROWS * 128;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const char* base = buf + (long)(blockIdx.x % 64) * panel;
  uint32_t off[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int lin = (w * NI + i) * 64 + lane, row = lin >> 3, ch = lin & 7;
    off[i] = (uint32_t)(row * stride + ch * 16);
  }
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) char*)smem + (uint32_t)(w * NI * 1024);
  auto load = [&](int s, int slot) {
    const uint64_t b = (uint64_t)(uintptr_t)(base + (long)(s & 15) * 128);
    const uint64_t sb = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t l = lds0 + (uint32_t)(slot * STAGE);
#pragma unroll
    for (int i = 0; i < NI; i += 2) glds16x2(sb, off[i], off[i + 1], l + i * 1024, l + (i + 1) * 1024);
  };
  for (int s = 0; s < NSTAGE - 1; ++s) load(s, s);
  int slot = 0;
  for (int s = 0; s < steps; ++s) {
    const int ahead = min(steps - 1 - s, NSTAGE - 2);
    if (ahead >= NSTAGE - 2) wait_vm<(NSTAGE - 2) * NI>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    if (s + NSTAGE - 1 < steps) load(s + NSTAGE - 1, slot == 0 ? NSTAGE - 1 : slot - 1);
    slot = slot == NSTAGE - 1 ? 0 : slot + 1;
  }
  wait_vm<0>();
  __syncthreads();
  if (tid == 0) sink[blockIdx.x] = smem[lane];
}

template <int ROWS, int DEPTH, bool WRITE>
__global__ __launch_bounds__(256, 1) void probe_reg(const char* buf, long stride, long panel, int steps,
                                                   int* sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NI = ROWS * 8 / 256;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const char* base = buf + (long)(blockIdx.x % 64) * panel;
  uint4 r[DEPTH][NI];
  uint4 x = make_uint4(0, 0, 0, 0);
  auto load = [&](int s, uint4 (&d)[NI]) {
    const long koff = (long)(s & 15) * 128;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int lin = (w * NI + i) * 64 + lane, row = lin >> 3, ch = lin & 7;
      d[i] = *(const uint4*)(base + row * stride + koff + ch * 16);
    }
  };
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) load(d, r[d]);
  for (int s = 0; s < steps; s += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        if constexpr (WRITE) {
          *(uint4*)(smem + ((d & 1) * NI + i) * 4096 + tid * 16) = r[d][i];
        } else {
          x.x ^= r[d][i].x; x.y ^= r[d][i].y; x.z ^= r[d][i].z; x.w ^= r[d][i].w;
        }
      }
      if (s + d + DEPTH < steps) load(s + d + DEPTH, r[d]);
    }
    if constexpr (WRITE) __builtin_amdgcn_s_barrier();
  }
  if constexpr (WRITE) {
    __syncthreads();
    x.x = *(const uint32_t*)(smem + tid * 4);
  }
  if (x.x == 0x12345678u) sink[blockIdx.x] = x.y + x.z + x.w;
}

typedef void (*KFn)(const char*, long, long, int, int*);

static float run(KFn k, int grid, size_t smem, const char* buf, long stride, long panel, int steps, int* sink) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  if (smem) CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(256), smem, 0, buf, stride, panel, steps, sink);
  CK(hipDeviceSynchronize());
  const int reps = 20;
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(256), smem, 0, buf, stride, panel, steps, sink);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipGetLastError());
  return ms / reps * 1e3f;   // us
}

int main() {
  const size_t bytes = 256u << 20;
  char* buf;
  int* sink;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&sink, 4096 * sizeof(int)));
  CK(hipMemset(buf, 1, bytes));
  const int grid = 256, steps = 256;
  struct S { long stride; const char* tag; };
  const S strides[] = {{2048, "2KB"}, {2048 + 128, "2KB+128"}, {8192, "8KB"}, {8192 + 128, "8KB+128"}, {6144, "6KB"}};
  for (const S& st : strides) {
    // 64 distinct 192-row panels spread over the buffer: panel = 192 rows * stride (L2-resident per XCD
    // when the whole set fits: 64 * 192 * stride bytes; at 2 KB that is 24 MB total, 3 MB per XCD)
    const long panel = 192 * st.stride / 8;     // panels overlap: 8 workgroups share rows -> L2 reuse
    struct V { KFn k; size_t smem; int rows; const char* name; };
    const V vs[] = {
        {probe_dma<192, 4>, 4 * 192 * 128, 192, "dma  rows192 nstage4"},
        {probe_dma<192, 6>, 6 * 192 * 128, 192, "dma  rows192 nstage6"},
        {probe_dma<128, 8>, 8 * 128 * 128, 128, "dma  rows128 nstage8"},
        {probe_dma<256, 4>, 4 * 256 * 128, 256, "dma  rows256 nstage4"},
        {probe_dma_sv<192, 4>, 4 * 192 * 128, 192, "dma-sv rows192 nstage4"},
        {probe_dma_sv<192, 6>, 6 * 192 * 128, 192, "dma-sv rows192 nstage6"},
        {probe_dma_sv<128, 8>, 8 * 128 * 128, 128, "dma-sv rows128 nstage8"},
        {probe_dma_sv<256, 4>, 4 * 256 * 128, 256, "dma-sv rows256 nstage4"},
        {probe_reg<192, 2, false>, 0, 192, "reg  rows192 depth2"},
        {probe_reg<192, 4, false>, 0, 192, "reg  rows192 depth4"},
        {probe_reg<128, 6, false>, 0, 128, "reg  rows128 depth6"},
        {probe_reg<192, 4, true>, 2 * 6 * 4096, 192, "reg+ds_write rows192 depth4"},
    };
    for (const V& v : vs) {
      const float us = run(v.k, grid, v.smem, buf, st.stride, panel, steps, sink);
      const double per_cu = (double)v.rows * 128 * steps / (us * 1e-6);
      printf("stride %-8s %-28s %8.1f us  %6.1f GB/s per workgroup  %6.2f TB/s total\n", st.tag, v.name, us,
             per_cu / 1e9, per_cu * grid / 1e12);
      fflush(stdout);
    }
  }
  // VERDICT r3 Weak #6: more workgroups per CU (2 and 4 resident: 8-16 waves) -- does the per-CU
  // rate rise above the one-workgroup figure, or is ~32 TB/s the L2's aggregate ceiling?
  for (int grid2 : {512, 1024}) {
    const long stride = 8192, panel = 192 * stride / 8;
    struct V { KFn k; size_t smem; int rows; const char* name; };
    const V vs[] = {
        {probe_dma<128, 4>, 4 * 128 * 128, 128, "dma  rows128 nstage4"},
        {probe_reg<192, 4, false>, 0, 192, "reg  rows192 depth4"},
        {probe_reg<128, 6, false>, 0, 128, "reg  rows128 depth6"},
    };
    for (const V& v : vs) {
      const float us = run(v.k, grid2, v.smem, buf, stride, panel, steps, sink);
      const double per_wg = (double)v.rows * 128 * steps / (us * 1e-6);
      printf("grid %4d (%d per CU) stride 8KB %-24s %8.1f us  %6.1f GB/s per CU  %6.2f TB/s total\n", grid2,
             grid2 / 256, v.name, us, per_wg * grid2 / 256 / 1e9, per_wg * grid2 / 1e12);
      fflush(stdout);
    }
  }
  return 0;
}
