// Fused AdamW over flat fp32 optimizer shards + gradient-norm helpers for gfx950.
//
// Replaces torch.optim.AdamW(foreach) (train_harness.py:329) and DeepSpeed's FusedAdam
// multi_tensor_adam for the ZeRO paths.  All optimizer state lives in ONE flat fp32 "owner"
// space per rank (the whole model for DDP, this rank's partition for ZeRO/FSDP), so a single
// launch updates master weights, exp_avg and exp_avg_sq in one HBM pass and writes the bf16
// compute copy of every parameter straight into its (possibly non-contiguous) destination:
//
//   segments: owner range [ostart, ostart + len) -> bf16 destination pointer
//   blocks  : host-built table (segment id, owner start) so no block straddles a segment.
//
// Math is torch.optim.AdamW's:  p *= 1 - lr*wd;  m = lerp(m, g, 1-b1);  v = b2 v + (1-b2) g^2;
//                                p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
// with g optionally multiplied by a device-side scale (gradient clipping coefficient / 1/accum),
// read from memory so no host sync is needed.
#include <cstdlib>

#include "common.h"

namespace {

constexpr int kAdamThreads = 256;
constexpr int kAdamChunk = kAdamThreads * 16;   // elements per block (host block tables)

typedef float v4f __attribute__((ext_vector_type(4)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

template <typename G>
DLTB_DEV void load4(const G* p, float* g);
template <>
DLTB_DEV void load4<float>(const float* p, float* g) {
  float4 v = *reinterpret_cast<const float4*>(p);
  g[0] = v.x; g[1] = v.y; g[2] = v.z; g[3] = v.w;
}
template <>
DLTB_DEV void load4<bf16_t>(const bf16_t* p, float* g) {
  uint2 v = *reinterpret_cast<const uint2*>(p);
  g[0] = lo_bf(v.x); g[1] = hi_bf(v.x); g[2] = lo_bf(v.y); g[3] = hi_bf(v.y);
}
// 8 gradient elements: one 16-byte load for 16-bit gradients, two for fp32
template <typename G>
DLTB_DEV void load8(const G* p, float* g);
template <>
DLTB_DEV void load8<float>(const float* p, float* g) {
  const v4f a = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p));
  const v4f b = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p + 4));
  g[0] = a[0]; g[1] = a[1]; g[2] = a[2]; g[3] = a[3]; g[4] = b[0]; g[5] = b[1]; g[6] = b[2]; g[7] = b[3];
}
template <>
DLTB_DEV void load8<bf16_t>(const bf16_t* p, float* g) {
  const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
  g[0] = lo_bf(v[0]); g[1] = hi_bf(v[0]); g[2] = lo_bf(v[1]); g[3] = hi_bf(v[1]);
  g[4] = lo_bf(v[2]); g[5] = hi_bf(v[2]); g[6] = lo_bf(v[3]); g[7] = hi_bf(v[3]);
}

struct AdamHp {
  float lr, beta1, beta2, eps, wd, step_size, inv_sqrt_bc2, gs;
};

DLTB_DEV void adam_elem(float& p, float& m, float& v, float g, const AdamHp& h) {
  const float gg = g * h.gs;
  p *= 1.f - h.lr * h.wd;
  m = m + (1.f - h.beta1) * (gg - m);
  v = h.beta2 * v + (1.f - h.beta2) * gg * gg;
  const float denom = sqrtf(v) * h.inv_sqrt_bc2 + h.eps;
  p -= h.step_size * m / denom;
}

// W elements per lane and vector access (8: every stream moved in 16-byte accesses -- master /
// moments as two float4, a 16-bit gradient and the 16-bit parameter copy as one 16-byte access;
// 4: the 8-byte 16-bit accesses of segments not 8-element aligned).  ITERS vectors per lane, all
// loads issued before the first update (ITERS * (6 + 1) 16-byte loads in flight per lane at W = 8).
template <typename G, int W, int T = kAdamThreads>
DLTB_DEV void adamw_block(float* __restrict__ master, float* __restrict__ exp_avg, float* __restrict__ exp_avg_sq,
                          const G* __restrict__ grad, bf16_t* __restrict__ dst, int64_t start, int64_t seg_end,
                          int64_t dst_base, const AdamHp& h) {
  constexpr int ITERS = kAdamChunk / (T * W);
  constexpr int NV = W / 4;
  v4f P[ITERS][NV], M[ITERS][NV], V[ITERS][NV];
  float Gr[ITERS][W];
#pragma unroll
  for (int it = 0; it < ITERS; ++it) {
    const int64_t i = start + ((int64_t)it * T + threadIdx.x) * W;
    if (i < seg_end) {
#pragma unroll
      for (int q = 0; q < NV; ++q) {
        P[it][q] = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(master + i + 4 * q));
        M[it][q] = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(exp_avg + i + 4 * q));
        V[it][q] = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(exp_avg_sq + i + 4 * q));
      }
      if constexpr (W == 8) load8<G>(grad + i, Gr[it]);
      else load4<G>(grad + i, Gr[it]);
    }
  }
#pragma unroll
  for (int it = 0; it < ITERS; ++it) {
    const int64_t off = ((int64_t)it * T + threadIdx.x) * W;
    const int64_t i = start + off;
    if (i >= seg_end) break;
    float p[W], m[W], v[W];
#pragma unroll
    for (int e = 0; e < W; ++e) {
      p[e] = P[it][e >> 2][e & 3];
      m[e] = M[it][e >> 2][e & 3];
      v[e] = V[it][e >> 2][e & 3];
      adam_elem(p[e], m[e], v[e], Gr[it][e], h);
    }
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      __builtin_nontemporal_store((v4f){p[4 * q], p[4 * q + 1], p[4 * q + 2], p[4 * q + 3]},
                                  reinterpret_cast<v4f*>(master + i + 4 * q));
      __builtin_nontemporal_store((v4f){m[4 * q], m[4 * q + 1], m[4 * q + 2], m[4 * q + 3]},
                                  reinterpret_cast<v4f*>(exp_avg + i + 4 * q));
      __builtin_nontemporal_store((v4f){v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]},
                                  reinterpret_cast<v4f*>(exp_avg_sq + i + 4 * q));
    }
    if constexpr (W == 8) {
      v4u o = {pack_bf2(p[0], p[1]), pack_bf2(p[2], p[3]), pack_bf2(p[4], p[5]), pack_bf2(p[6], p[7])};
      *reinterpret_cast<v4u*>(dst + dst_base + off) = o;
    } else {
      uint2 o;
      o.x = pack_bf2(p[0], p[1]);
      o.y = pack_bf2(p[2], p[3]);
      *reinterpret_cast<uint2*>(dst + dst_base + off) = o;
    }
  }
}

template <typename G>
__global__ __launch_bounds__(kAdamThreads) void adamw_kernel(
    float* __restrict__ master, float* __restrict__ exp_avg, float* __restrict__ exp_avg_sq,
    const G* __restrict__ grad, const int* __restrict__ blk_seg, const int64_t* __restrict__ blk_start,
    const int64_t* __restrict__ seg_ostart, const int64_t* __restrict__ seg_len,
    const int64_t* __restrict__ seg_dst, const float* __restrict__ gscale, const float* __restrict__ hp,
    float lr, float beta1, float beta2, float eps, float wd, float step_size, float inv_sqrt_bc2, int nblk) {
  if (hp) {   // step-dependent hyper-parameters from device memory (HIP-graph replays)
    if (hp[3] != 0.f) return;   // dynamic loss scaling found an inf / nan: the step is skipped
    lr = hp[0];
    step_size = hp[1];
    inv_sqrt_bc2 = hp[2];
  }
  // one table row per block, or (a grid capped below the row count: an update trickled beside other
  // kernels) a block-strided walk over the rows
  for (int bi = blockIdx.x; bi < nblk; bi += gridDim.x) {
  const int seg = blk_seg[bi];
  const int64_t start = blk_start[bi];
  const int64_t s0 = seg_ostart[seg];
  const int64_t seg_end = s0 + seg_len[seg];
  DLTB_DCHECK(seg >= 0 && start >= s0 && start < seg_end);
  bf16_t* dst = reinterpret_cast<bf16_t*>(seg_dst[seg]);
  const int64_t dst_base = start - s0;
  const AdamHp h{lr, beta1, beta2, eps, wd, step_size, inv_sqrt_bc2, gscale ? *gscale : 1.f};
  // every state element is touched once per step: streamed past the caches (nontemporal loads and
  // stores).  W = 4: every fp32 access one coalesced 16-byte vector per lane, the 16-bit streams 8 bytes
  // per lane (a W = 8 path -- two adjacent float4 per lane -- measured 4.22 TB/s against 5.52 on the
  // TinyGPT-A state, and 128-thread blocks no faster: profiles/adamw_r5.txt; both removed in round 6).
  adamw_block<G, 4>(master, exp_avg, exp_avg_sq, grad, dst, start, seg_end, dst_base, h);
  }
}

// sum of squares in a FIXED order (bitwise reproducible: eager runs, graph replays and ranks agree):
// a grid-stride pass writes one partial per block, a one-block pass adds them in index order.
constexpr int kSumsqBlocks = 1024;

template <typename G>
__global__ __launch_bounds__(256) void sumsq_kernel(const G* __restrict__ x, long n4,
                                                   float* __restrict__ part) {
  __shared__ float red[4];
  // four grid-strided loads issued before any is consumed (four independent accumulators): the
  // pass is HBM-latency bound with one 8-byte load in flight per lane
  const long stride = (long)gridDim.x * blockDim.x;
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  for (; i + 3 * stride < n4; i += 4 * stride) {
    float g[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) load4<G>(x + (i + u * stride) * 4, g[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] += g[u][0] * g[u][0] + g[u][1] * g[u][1] + g[u][2] * g[u][2] + g[u][3] * g[u][3];
  }
  for (; i < n4; i += stride) {
    float g[4];
    load4<G>(x + i * 4, g);
    a[0] += g[0] * g[0] + g[1] * g[1] + g[2] * g[2] + g[3] * g[3];
  }
  float acc = (a[0] + a[1]) + (a[2] + a[3]);
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

__global__ __launch_bounds__(256) void sumsq_final_kernel(const float* __restrict__ part, int n,
                                                         float* __restrict__ out) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) acc += part[i];
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) out[0] += acc;
}

// norm_sq[0] (already all-reduced) -> coef = min(1, max_norm / (sqrt(norm_sq) + 1e-6)), norm
__global__ void clip_coef_kernel(const float* __restrict__ norm_sq, float max_norm,
                                 float* __restrict__ coef, float* __restrict__ norm_out,
                                 float extra_scale) {
  const float nrm = sqrtf(norm_sq[0]) * extra_scale;
  float c = max_norm > 0.f ? max_norm / (nrm + 1e-6f) : 1.f;
  c = fminf(c, 1.f);
  coef[0] = c * extra_scale;
  if (norm_out) norm_out[0] = nrm;
}

// Dynamic loss scaling with torch.amp.GradScaler's semantics (train_harness.py:334-335, 371-376),
// decided on the device so no step ever waits on the host:
//   state = [scale S, growth tracker, optimizer steps taken, steps skipped]
//   norm_sq = sum of squares of the S-scaled gradients (all-reduced where sharded); an inf or nan
//   gradient makes it non-finite (fp16 gradients cannot overflow the fp32 sum: 65504^2 * 2^28).
// found inf -> hp[3] = 1 (the AdamW kernel returns at once: master, moments and step count stay),
//              S *= backoff, tracker = 0;
// otherwise -> coef = extra * clip(unscaled norm) / S, hp[1..2] = bias corrections of the device
//              step count, tracker += 1, S *= growth when it reaches growth_interval.
// hp[0] (lr) is the host's upload (FlatAdamW.prepare) and is left alone.
__global__ void amp_step_kernel(const float* __restrict__ norm_sq, float* __restrict__ state,
                                float* __restrict__ coef, float* __restrict__ norm_out,
                                float* __restrict__ hp, float max_norm, float extra_scale, float beta1,
                                float beta2, float growth, float backoff, float growth_interval) {
  const float S = state[0];
  const float nsq = norm_sq[0];
  if (!isfinite(nsq)) {
    state[0] = S * backoff;
    state[1] = 0.f;
    state[3] += 1.f;
    hp[3] = 1.f;
    coef[0] = 0.f;
    if (norm_out) norm_out[0] = nsq;
    return;
  }
  const float inv = 1.f / S;
  const float nrm = sqrtf(nsq) * inv * extra_scale;
  const float c = max_norm > 0.f ? fminf(1.f, max_norm / (nrm + 1e-6f)) : 1.f;
  coef[0] = c * extra_scale * inv;
  if (norm_out) norm_out[0] = nrm;
  const float t = state[2] + 1.f;
  state[2] = t;
  hp[1] = hp[0] / (1.f - powf(beta1, t));
  hp[2] = 1.f / sqrtf(1.f - powf(beta2, t));
  hp[3] = 0.f;
  float tr = state[1] + 1.f;
  if (tr >= growth_interval) {
    state[0] = S * growth;
    tr = 0.f;
  }
  state[1] = tr;
}

__global__ __launch_bounds__(256) void fill_f32_kernel(float* __restrict__ x, long n, float v) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    x[i] = v;
}

}  // namespace

int dltb_adamw_chunk() { return kAdamChunk; }

void dltb_adamw(float* master, float* exp_avg, float* exp_avg_sq, const void* grad, bool grad_bf16,
                const int* blk_seg, const int64_t* blk_start, int nblocks, const int64_t* seg_ostart,
                const int64_t* seg_len, const int64_t* seg_dst, const float* gscale, const float* hp,
                float lr, float beta1, float beta2, float eps, float wd, float step_size,
                float inv_sqrt_bc2, int grid_cap, hipStream_t st) {
  if (nblocks <= 0) return;
  const int grid = grid_cap > 0 && grid_cap < nblocks ? grid_cap : nblocks;
  const int thr = kAdamThreads;
  if (grad_bf16)
    hipLaunchKernelGGL(adamw_kernel<bf16_t>, dim3(grid), dim3(thr), 0, st, master,
                       exp_avg, exp_avg_sq, (const bf16_t*)grad, blk_seg, blk_start, seg_ostart,
                       seg_len, seg_dst, gscale, hp, lr, beta1, beta2, eps, wd, step_size, inv_sqrt_bc2, nblocks);
  else
    hipLaunchKernelGGL(adamw_kernel<float>, dim3(grid), dim3(thr), 0, st, master,
                       exp_avg, exp_avg_sq, (const float*)grad, blk_seg, blk_start, seg_ostart,
                       seg_len, seg_dst, gscale, hp, lr, beta1, beta2, eps, wd, step_size, inv_sqrt_bc2, nblocks);
}

int dltb_sumsq_partials() { return kSumsqBlocks; }

void dltb_sumsq(const void* x, bool bf16, long n, float* out, float* part, hipStream_t st) {
  const long n4 = n / 4;
  long g = (n4 + 255) / 256;
  if (g > kSumsqBlocks) g = kSumsqBlocks;
  if (g < 1) g = 1;
  if (bf16)
    hipLaunchKernelGGL(sumsq_kernel<bf16_t>, dim3(g), dim3(256), 0, st, (const bf16_t*)x, n4, part);
  else
    hipLaunchKernelGGL(sumsq_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)x, n4, part);
  hipLaunchKernelGGL(sumsq_final_kernel, dim3(1), dim3(256), 0, st, part, (int)g, out);
}

void dltb_clip_coef(const float* norm_sq, float max_norm, float* coef, float* norm_out,
                    float extra_scale, hipStream_t st) {
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(1), 0, st, norm_sq, max_norm, coef, norm_out,
                     extra_scale);
}

void dltb_amp_step(const float* norm_sq, float* state, float* coef, float* norm_out, float* hp,
                   float max_norm, float extra_scale, float beta1, float beta2, float growth,
                   float backoff, int growth_interval, hipStream_t st) {
  hipLaunchKernelGGL(amp_step_kernel, dim3(1), dim3(1), 0, st, norm_sq, state, coef, norm_out, hp,
                     max_norm, extra_scale, beta1, beta2, growth, backoff, (float)growth_interval);
}

void dltb_fill_f32(float* x, long n, float v, hipStream_t st) {
  long g = (n + 255) / 256;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(fill_f32_kernel, dim3(g), dim3(256), 0, st, x, n, v);
}
