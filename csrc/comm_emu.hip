// Emulated-fabric collective: the stand-in for one RCCL collective of an N-rank job, run by a single
// process on one MI355X (DLTB_COMM=emulate:N, comm/collectives.py).
//
// A real RCCL collective on an 8 x MI355X node is a kernel of `channels` workgroups that, for the
// collective's duration, occupies those CUs and streams the buffer through HBM while the bytes cross
// xGMI.  This kernel reproduces exactly those three things for the compute that runs beside it:
//   * occupancy: `channels` workgroups of 512 threads stay resident until the modelled end time;
//   * HBM traffic: it reads the collective's buffer (`traffic`, `passes` times) and writes the
//     stand-in result;
//   * duration: every wave paces itself against the 100 MHz constant wall clock so that its share
//     of the work finishes no earlier than t0 + alpha + beta * (fraction done), where alpha / beta
//     come from the alpha-beta model of comm/topology.py (fixed latency, wire bytes / bus
//     bandwidth).  Waiting waves sleep (s_sleep), so they cost issue slots only when they poll.
// If the memory work is slower than the pace (a contended HBM) the kernel simply runs longer, as
// a real collective would.
//
// Numerics stand-in (the data a rank would hold afterwards if every rank held the same data):
//   dst[r * rep_stride + j] = scale * src[j]   for r < replicas, j < n     (scale 1: plain copy)
// reduce-scatter: dst = own chunk, src = own chunk of the input, scale = N; all-reduce (sum): in
// place, scale = N; all-gather into a separate buffer: replicas = N copies of the local shard.
#include "common.h"
#include "launchers.h"

#include <stdexcept>

namespace {

constexpr int kThreads = 512;

struct EmuArgs {
  const uint4* traffic;   // buffer streamed to model the collective's HBM reads
  long traffic_vec;       // 16-byte vectors per pass
  int passes;
  uint4* dst;
  const uint4* src;
  long n_vec;             // 16-byte vectors of the numerics stand-in (per replica)
  int f32;                // element type of dst / src: fp32 (1) or this object's 16-bit format (0)
  float scale;
  int replicas;
  long rep_stride_vec;
  long alpha_ticks;       // fixed latency, wall-clock ticks
  long beta_ticks;        // bandwidth term, wall-clock ticks
  uint32_t magic;         // never equal to the traffic checksum in practice: keeps the loads alive
  uint32_t* sink;
};

DLTB_DEV uint64_t now() { return wall_clock64(); }

DLTB_DEV void pace_until(uint64_t target) {
  while (now() < target) __builtin_amdgcn_s_sleep(8);
}

DLTB_DEV uint4 scaled(uint4 v, float s, int f32) {
  if (s == 1.f) return v;
  if (f32) {
    float4 f = __builtin_bit_cast(float4, v);
    f.x *= s; f.y *= s; f.z *= s; f.w *= s;
    return __builtin_bit_cast(uint4, f);
  }
  float f[8];
  unpack8(v, f);
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] *= s;
  return pack8(f);
}

// One tile = kThreads x kVec 16-byte vectors (128 KiB): every lane has kVec independent loads in
// flight before it consumes any, so 32 workgroups can stream the buffer well above the modelled
// fabric rate and the pace, not the loop, sets the duration (measured: tests/test_emulate_gpu.py).
constexpr int kVec = 16;
constexpr long kTile = (long)kThreads * kVec;

__global__ __launch_bounds__(kThreads) void comm_emu_kernel(EmuArgs a) {
  const uint64_t t0 = now();
  const long n_num = a.n_vec * a.replicas, n_trf = a.traffic_vec * a.passes;
  const long num_tiles = (n_num + kTile - 1) / kTile;
  const long tiles = num_tiles + (n_trf + kTile - 1) / kTile;
  const long G = gridDim.x;
  const long mine = tiles > blockIdx.x ? (tiles - blockIdx.x + G - 1) / G : 0;
  uint32_t acc = 0;
  long k = 0;
  for (long t = blockIdx.x; t < tiles; t += G, ++k) {
    if (t < num_tiles) {
      uint4 v[kVec];
      long e[kVec];
#pragma unroll
      for (int u = 0; u < kVec; ++u) {                      // element vectors over (replica, j)
        e[u] = t * kTile + u * kThreads + threadIdx.x;
        if (e[u] < n_num) v[u] = a.src[e[u] % a.n_vec];
      }
#pragma unroll
      for (int u = 0; u < kVec; ++u)
        if (e[u] < n_num) {
          const long r = e[u] / a.n_vec, j = e[u] - r * a.n_vec;
          a.dst[r * a.rep_stride_vec + j] = scaled(v[u], a.scale, a.f32);
        }
    } else {
      uint4 v[kVec];
#pragma unroll
      for (int u = 0; u < kVec; ++u) {
        const long e = (t - num_tiles) * kTile + u * kThreads + threadIdx.x;
        v[u] = e < n_trf ? a.traffic[e % a.traffic_vec] : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < kVec; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    // the modelled time at which this workgroup's first k + 1 tiles are done
    pace_until(t0 + a.alpha_ticks + (uint64_t)((double)a.beta_ticks * (double)(k + 1) / (double)mine));
  }
  pace_until(t0 + a.alpha_ticks + a.beta_ticks);
  if (acc == a.magic) a.sink[threadIdx.x] = acc;
}

// tiny or unaligned buffers (the one-float grad-norm all-reduce): one lane per element
__global__ void comm_emu_scalar_kernel(void* dst, const void* src, long n, int f32, float scale, int replicas,
                                       long rep_stride, long ticks) {
  const uint64_t t0 = now();
  for (long e = threadIdx.x; e < n * replicas; e += blockDim.x) {
    const long r = e / n, j = e - r * n;
    if (f32) {
      static_cast<float*>(dst)[r * rep_stride + j] = scale * static_cast<const float*>(src)[j];
    } else {
      const float v = bf2f(static_cast<const bf16_t*>(src)[j]);
      static_cast<bf16_t*>(dst)[r * rep_stride + j] = f2bf(scale * v);
    }
  }
  pace_until(t0 + ticks);
}

double ticks_per_us() {
  static double t = [] {
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
    return khz / 1000.0;
  }();
  return t;
}

uint32_t* sink_buffer() {
  static uint32_t* s = [] {
    void* p = nullptr;
    if (hipMalloc(&p, kThreads * sizeof(uint32_t)) != hipSuccess) throw std::runtime_error("comm_emu sink alloc");
    return static_cast<uint32_t*>(p);
  }();
  return s;
}

}  // namespace

void dltb_comm_emu(const void* traffic, long traffic_bytes, int passes, void* dst, const void* src, long n,
                   int elem, float scale, int replicas, long rep_stride, float alpha_us, float beta_us,
                   int channels, hipStream_t st) {
  const double tpu = ticks_per_us();
  const long alpha = (long)(alpha_us * tpu), beta = (long)(beta_us * tpu);
  const bool vec = n > 0 && (n * elem) % 16 == 0 && (rep_stride * elem) % 16 == 0 &&
                   (reinterpret_cast<uintptr_t>(dst) % 16) == 0 && (reinterpret_cast<uintptr_t>(src) % 16) == 0;
  if (!vec && n > 0) {       // small: numerics by one workgroup, the whole duration paced there
    comm_emu_scalar_kernel<<<1, 64, 0, st>>>(dst, src, n, elem == 4, scale, replicas, rep_stride, alpha + beta);
    return;
  }
  EmuArgs a;
  a.traffic = static_cast<const uint4*>(traffic);
  a.traffic_vec = traffic ? traffic_bytes / 16 : 0;
  a.passes = passes > 0 ? passes : 1;
  a.dst = static_cast<uint4*>(dst);
  a.src = static_cast<const uint4*>(src);
  a.n_vec = n > 0 ? n * elem / 16 : 0;
  a.f32 = elem == 4;
  a.scale = scale;
  a.replicas = replicas > 0 ? replicas : 1;
  a.rep_stride_vec = rep_stride * elem / 16;
  a.alpha_ticks = alpha;
  a.beta_ticks = beta;
  a.magic = 0x9E3779B9u;
  a.sink = sink_buffer();
  comm_emu_kernel<<<channels > 0 ? channels : 1, kThreads, 0, st>>>(a);
}
