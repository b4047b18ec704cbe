// LayerNorm / RMSNorm forward + backward for gfx950.
//
// Forward (optionally fused with the residual add + dropout that precedes it):
//     s = x + dropout(r)          (HAS_RES; s is written in bf16 and is the residual stream)
//     y = (s - mean) * rstd * w + b          (LayerNorm)   |   y = s * rstd * w   (RMSNorm)
// One 64-lane wave per row, the row held in registers as 16-byte bf16x8 vectors, fp32 stats.
//
// Backward: one wave per row computes dx (+ the incoming residual gradient) and accumulates
// per-column dgamma/dbeta partials; a block folds its 4 waves through LDS float atomics and
// writes one fp32 partial row; `norm_colreduce` sums the partials into the bf16 gradient slot
// (overwrite or accumulate).  Reference ops: nn.LayerNorm (train_harness.py:112,117,56).
#include "attn_mask.h"
#include "common.h"

namespace {

constexpr int kRowsPerWave = 4;   // backward: rows per wave
constexpr int kWaves = 4;

// one wave = one row (the body of norm_fwd_kernel and of norm_fwd_mask_kernel's norm blocks)
template <int NV, bool RMS, bool HAS_RES>
DLTB_DEV void norm_fwd_row(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ r, const bf16_t* __restrict__ w,
    const bf16_t* __restrict__ b, bf16_t* __restrict__ s_out, bf16_t* __restrict__ y,
    float* __restrict__ mean_out, float* __restrict__ rstd_out, int N, int d, float eps,
    uint32_t thr16, float drop_scale, const int64_t* __restrict__ seed_ptr, int64_t site, int row, int lane) {
  if (row >= N) return;
  const int nvec = d >> 3;
  const size_t base = (size_t)row * d;
  float v[NV][8];
  uint64_t seed = 0;
  uint32_t rk = 0;
  const bool do_drop = HAS_RES && thr16 > 0;
  if (do_drop) {
    seed = site_seed(seed_ptr, site);
    rk = rng_row_key(seed, (uint32_t)row);
  }
  uint4 wraw[NV], braw[NV];           // weight / bias issued first: their latency hides under the stats
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int idx = j * 64 + lane;
    if (idx < nvec) {
      wraw[j] = ld16<uint4>(w + idx * 8);
      if (!RMS) braw[j] = ld16<uint4>(b + idx * 8);
    }
  }
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int idx = j * 64 + lane;
    if (idx < nvec) {
      uint4 xv = ld16<uint4>(x + base + idx * 8);
      unpack8(xv, v[j]);
      if (HAS_RES) {
        float rv[8];
        unpack8(ld16<uint4>(r + base + idx * 8), rv);
        if (do_drop) {
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            const uint32_t col = (uint32_t)(idx * 8 + e);
            const uint32_t hsh = rng_pair(rk, rng_col_key(seed, col));
            rv[e] = keep_lo(hsh, thr16) ? rv[e] * drop_scale : 0.f;
            rv[e + 1] = keep_hi(hsh, thr16) ? rv[e + 1] * drop_scale : 0.f;
          }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) v[j][e] = bf2f(f2bf(v[j][e] + rv[e]));  // round like the stored s
        *reinterpret_cast<uint4*>(s_out + base + idx * 8) = pack8(v[j]);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) sum += v[j][e];
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[j][e] = 0.f;
    }
  }
  float mean = 0.f;
  if (!RMS) mean = wave_sum(sum) / (float)d;
  float sq = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int idx = j * 64 + lane;
    if (idx < nvec) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float c = v[j][e] - mean;
        sq += c * c;
      }
    }
  }
  const float var = wave_sum(sq) / (float)d;
  const float rstd = rsqrtf(var + eps);
  if (lane == 0) {
    if (!RMS) mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int idx = j * 64 + lane;
    if (idx < nvec) {
      float wv[8], o[8];
      unpack8(wraw[j], wv);
      if (!RMS) {
        float bv[8];
        unpack8(braw[j], bv);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (v[j][e] - mean) * rstd * wv[e] + bv[e];
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = v[j][e] * rstd * wv[e];
      }
      *reinterpret_cast<uint4*>(y + base + idx * 8) = pack8(o);
    }
  }
}

template <int NV, bool RMS, bool HAS_RES>
__global__ __launch_bounds__(256) void norm_fwd_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ r, const bf16_t* __restrict__ w,
    const bf16_t* __restrict__ b, bf16_t* __restrict__ s_out, bf16_t* __restrict__ y,
    float* __restrict__ mean_out, float* __restrict__ rstd_out, int N, int d, float eps,
    uint32_t thr16, float drop_scale, const int64_t* __restrict__ seed_ptr, int64_t site) {
  norm_fwd_row<NV, RMS, HAS_RES>(x, r, w, b, s_out, y, mean_out, rstd_out, N, d, eps, thr16, drop_scale,
                                 seed_ptr, site, blockIdx.x * kWaves + (threadIdx.x >> 6), threadIdx.x & 63);
}

// A block's first LayerNorm and its attention-dropout mask in ONE launch (horizontal fusion):
// blocks [0, nb_norm) are norm_fwd_kernel's blocks, the rest attn_mask_kernel's (flattened
// (query chunk, tile group) grid).  The mask hash is VALU-bound and the row norm waits on memory,
// so the two kinds of waves share the CUs instead of running back to back.
struct MaskJob {
  uint32_t* mask;
  int T;
  uint32_t thr16;
  const int64_t* seed;
  int64_t site;
  int gx;              // query chunks of 256 per tile group
  int g0;              // first tile group of this launch (a mask may be split over two launches)
};

template <int NV, bool RMS, bool HAS_RES>
__global__ __launch_bounds__(256) void norm_fwd_mask_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ r, const bf16_t* __restrict__ w,
    const bf16_t* __restrict__ b, bf16_t* __restrict__ s_out, bf16_t* __restrict__ y,
    float* __restrict__ mean_out, float* __restrict__ rstd_out, int N, int d, float eps,
    uint32_t thr16, float drop_scale, const int64_t* __restrict__ seed_ptr, int64_t site, int nb_norm,
    MaskJob mj) {
  const int bid = blockIdx.x;
  if (bid < nb_norm) {
    norm_fwd_row<NV, RMS, HAS_RES>(x, r, w, b, s_out, y, mean_out, rstd_out, N, d, eps, thr16, drop_scale,
                                   seed_ptr, site, bid * kWaves + (threadIdx.x >> 6), threadIdx.x & 63);
  } else {
    const int m = bid - nb_norm;
    attn_mask_word(mj.mask, mj.T, mj.thr16, mj.seed, mj.site, (m % mj.gx) * 256 + threadIdx.x,
                   (uint32_t)(mj.g0 + m / mj.gx));
  }
}

// dx: one wave per row, 4 rows per block (full occupancy); dy and s are read twice, the second
// pass hits L1/L2.
template <int NV, bool RMS, bool HAS_RES_GRAD>
__global__ __launch_bounds__(256) void norm_bwd_dx_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ s, const bf16_t* __restrict__ w,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    const bf16_t* __restrict__ dres, bf16_t* __restrict__ dx, int N, int d) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (row >= N) return;
  const int nvec = d >> 3;
  const size_t base = (size_t)row * d;
  const float mean = RMS ? 0.f : mean_in[row];
  const float rstd = rstd_in[row];
  float s1 = 0.f, s2 = 0.f;   // sum(w*dy), sum(w*dy*xhat)
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int idx = j * 64 + lane;
    if (idx < nvec) {
      float dyv[8], xv[8], wv[8];
      unpack8(ld16<uint4>(dy + base + idx * 8), dyv);
      unpack8(ld16<uint4>(s + base + idx * 8), xv);
      unpack8(ld16<uint4>(w + idx * 8), wv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float g = dyv[e] * wv[e];
        s1 += g;
        s2 += g * (xv[e] - mean) * rstd;
      }
    }
  }
  s1 = RMS ? 0.f : wave_sum(s1) / (float)d;
  s2 = wave_sum(s2) / (float)d;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int idx = j * 64 + lane;
    if (idx < nvec) {
      float dyv[8], xv[8], wv[8], o[8];
      unpack8(ld16<uint4>(dy + base + idx * 8), dyv);
      unpack8(ld16<uint4>(s + base + idx * 8), xv);
      unpack8(ld16<uint4>(w + idx * 8), wv);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = rstd * (dyv[e] * wv[e] - s1 - (xv[e] - mean) * rstd * s2);
      if (HAS_RES_GRAD) {
        float rv[8];
        unpack8(ld16<uint4>(dres + base + idx * 8), rv);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += rv[e];
      }
      *reinterpret_cast<uint4*>(dx + base + idx * 8) = pack8(o);
    }
  }
}

// Fused backward, one pass over dy / s: dx (+ the residual gradient) AND the fp32 column partials of
// dgamma = sum_r dy * xhat, dbeta = sum_r dy (LayerNorm only) and, with DXSUM, of the stored dx
// itself (the bias gradient of the linear whose output entered this residual stream).  Each wave
// owns `rpw` consecutive rows (one at TinyGPT's 2048 tokens) and keeps its column sums in registers;
// the 8 waves fold through one [8][d] LDS image, one partial at a time.  part: [K][gridDim.x][d]
// with K = (RMS ? 1 : 2) + DXSUM, summed into the gradient slots by colreduce_multi.  Replaces
// norm_bwd_dx + a colpart launch.
constexpr int kFusedWaves = 8;     // 512-thread blocks: two waves per SIMD at one block per CU
// one-barrier fold while the K x 8 x d fp32 images fit (d <= 1024 at K = 3): -0.4 us per launch isolated,
// profiles/norm_bwd_fold_ab_r6.txt
constexpr size_t kFoldLdsMax = 128 * 1024;

// XS (extra column sum): 0 none; 1 the stored dx; 2 the dropout backward of dx, dm = keep * dx / (1-p)
// with the keep bits of dropout site `site` (bitwise the colpart DROP kernel's dm), stored to `dm`,
// and its column sums -- the gradient of the previous block's MLP dropout and fc2 bias, produced
// here while dx is in registers (one colpart launch less per layer).
template <int NV, bool RMS, bool HAS_RES_GRAD, int XS>
__global__ __launch_bounds__(kFusedWaves * 64) void norm_bwd_fused_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ s, const bf16_t* __restrict__ w,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    const bf16_t* __restrict__ dres, bf16_t* __restrict__ dx, float* __restrict__ part, int N, int d,
    int rpw, bf16_t* __restrict__ dm, uint32_t thr16, float drop_scale, const int64_t* __restrict__ seed_ptr,
    int64_t site, bool one_fold) {
  // [kFusedWaves][d], or [K][kFusedWaves][d] with one_fold (all partial images folded after one barrier)
  extern __shared__ __attribute__((aligned(16))) float fold[];
  constexpr bool DXSUM = XS != 0;
  constexpr int K = (RMS ? 1 : 2) + (DXSUM ? 1 : 0);
  const uint64_t dseed = (XS == 2 && thr16) ? site_seed(seed_ptr, site) : 0ull;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nvec = d >> 3;
  float wv[NV][8], acc[K][NV][8];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int idx = j * 64 + lane;
    if (idx < nvec) unpack8(ld16<uint4>(w + idx * 8), wv[j]);
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[k][j][e] = 0.f;
  }
  const int r0 = (blockIdx.x * kFusedWaves + wid) * rpw;
  const int r1 = min(N, r0 + rpw);
  for (int row = r0; row < r1; ++row) {                  // wave-uniform trip count
    const size_t base = (size_t)row * d;
    const float mean = RMS ? 0.f : mean_in[row];
    const float rstd = rstd_in[row];
    float g[NV][8], xh[NV][8];
    float s1 = 0.f, s2 = 0.f;
    uint4 rraw[NV];                                      // residual gradient: issued with dy / s, so its
    if (HAS_RES_GRAD) {                                  // latency hides under the row reductions
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const int idx = j * 64 + lane;
        if (idx < nvec) rraw[j] = ld16<uint4>(dres + base + idx * 8);
      }
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int idx = j * 64 + lane;
      if (idx < nvec) {
        float dyv[8], xv[8];
        unpack8(ld16<uint4>(dy + base + idx * 8), dyv);
        unpack8(ld16<uint4>(s + base + idx * 8), xv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          xh[j][e] = (xv[e] - mean) * rstd;
          g[j][e] = dyv[e] * wv[j][e];
          s1 += g[j][e];
          s2 += g[j][e] * xh[j][e];
          acc[0][j][e] += dyv[e] * xh[j][e];
          if (!RMS) acc[1][j][e] += dyv[e];
        }
      }
    }
    s1 = RMS ? 0.f : wave_sum(s1) / (float)d;
    s2 = wave_sum(s2) / (float)d;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int idx = j * 64 + lane;
      if (idx < nvec) {
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = rstd * (g[j][e] - s1 - xh[j][e] * s2);
        if (HAS_RES_GRAD) {
          float rv[8];
          unpack8(rraw[j], rv);
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] += rv[e];
        }
        const uint4 ov = pack8(o);
        *reinterpret_cast<uint4*>(dx + base + idx * 8) = ov;
        if (DXSUM) {
          unpack8(ov, o);                                // sum the rounded dx the next GEMM reads
          if (XS == 2) {
            if (thr16) {
              const uint32_t rk = rng_row_key(dseed, (uint32_t)row);
#pragma unroll
              for (int e = 0; e < 8; e += 2) {
                const uint32_t hh = rng_pair(rk, rng_col_key(dseed, (uint32_t)(idx * 8 + e)));
                o[e] = keep_lo(hh, thr16) ? o[e] * drop_scale : 0.f;
                o[e + 1] = keep_hi(hh, thr16) ? o[e + 1] * drop_scale : 0.f;
              }
            }
            const uint4 mv = pack8(o);
            *reinterpret_cast<uint4*>(dm + base + idx * 8) = mv;
            unpack8(mv, o);                              // sum the rounded dm the fc2 GEMMs read
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[K - 1][j][e] += o[e];
        }
      }
    }
  }
  if (one_fold) {                                        // LDS holds all K images: one barrier
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const int idx = j * 64 + lane;
        if (idx < nvec) {
          float4* f = reinterpret_cast<float4*>(fold + (k * kFusedWaves + wid) * d + idx * 8);
          f[0] = make_float4(acc[k][j][0], acc[k][j][1], acc[k][j][2], acc[k][j][3]);
          f[1] = make_float4(acc[k][j][4], acc[k][j][5], acc[k][j][6], acc[k][j][7]);
        }
      }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k)
      for (int c = threadIdx.x; c < d; c += kFusedWaves * 64) {
        float t = 0.f;
#pragma unroll
        for (int v = 0; v < kFusedWaves; ++v) t += fold[(k * kFusedWaves + v) * d + c];
        part[((size_t)k * gridDim.x + blockIdx.x) * d + c] = t;
      }
    return;
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if (k) __syncthreads();                              // the previous partial has been read
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int idx = j * 64 + lane;
      if (idx < nvec) {
        float4* f = reinterpret_cast<float4*>(fold + wid * d + idx * 8);
        f[0] = make_float4(acc[k][j][0], acc[k][j][1], acc[k][j][2], acc[k][j][3]);
        f[1] = make_float4(acc[k][j][4], acc[k][j][5], acc[k][j][6], acc[k][j][7]);
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < d; c += kFusedWaves * 64) {
      float t = 0.f;
#pragma unroll
      for (int v = 0; v < kFusedWaves; ++v) t += fold[v * d + c];
      part[((size_t)k * gridDim.x + blockIdx.x) * d + c] = t;
    }
  }
}

// dgamma / dbeta column partials: block (bx, by) covers columns [bx*512, +512) and rows
// [by*rps, +rps); lane -> 8 columns, wave -> every 4th row.  part: [2][P][d]
template <bool RMS>
__global__ __launch_bounds__(256) void norm_dgamma_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ s, const float* __restrict__ mean_in,
    const float* __restrict__ rstd_in, float* __restrict__ part, int N, int d, int rps) {
  __shared__ __attribute__((aligned(16))) float red[2][4][512];
  const int lane = threadIdx.x & 63, phase = threadIdx.x >> 6;
  const int col = blockIdx.x * 512 + lane * 8;
  const int r0 = blockIdx.y * rps;
  const int r1 = min(N, r0 + rps);
  float ag[8], ab[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { ag[e] = 0.f; ab[e] = 0.f; }
  if (col < d) {
    for (int r = r0 + phase; r < r1; r += 4) {
      const size_t off = (size_t)r * d + col;
      const float mean = RMS ? 0.f : mean_in[r];
      const float rstd = rstd_in[r];
      float dyv[8], xv[8];
      unpack8(ld16<uint4>(dy + off), dyv);
      unpack8(ld16<uint4>(s + off), xv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        ag[e] += dyv[e] * (xv[e] - mean) * rstd;
        ab[e] += dyv[e];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[0][phase][lane * 8 + e] = ag[e];
    red[1][phase][lane * 8 + e] = ab[e];
  }
  __syncthreads();
  const int P = gridDim.y;
  for (int c = threadIdx.x; c < 512; c += 256) {
    const int gc = blockIdx.x * 512 + c;
    if (gc < d) {
      part[(size_t)blockIdx.y * d + gc] = red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c];
      if (!RMS)
        part[(size_t)(P + blockIdx.y) * d + gc] = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
    }
  }
}

// sum P partial rows -> bf16 (overwrite / accumulate); blockIdx.y selects (part0, out0) or
// (part0 + P*d, out1).  256 threads = 16 column quads x 16 row phases, float4 loads.
__global__ __launch_bounds__(256) void norm_colreduce_kernel(const float* __restrict__ part, int P,
                                                             int d, bf16_t* __restrict__ gw,
                                                             bf16_t* __restrict__ gb,
                                                             int accumulate) {
  __shared__ float red[16][65];
  const float* src = part + (size_t)blockIdx.y * P * d;
  bf16_t* out = blockIdx.y ? gb : gw;
  const int cq = threadIdx.x & 15, ph = threadIdx.x >> 4;
  const int c0 = blockIdx.x * 64 + cq * 4;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c0 < d) {
    for (int p = ph; p < P; p += 16) {
      const float4 v = *reinterpret_cast<const float4*>(src + (size_t)p * d + c0);
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
  }
  red[ph][cq * 4 + 0] = a.x;
  red[ph][cq * 4 + 1] = a.y;
  red[ph][cq * 4 + 2] = a.z;
  red[ph][cq * 4 + 3] = a.w;
  __syncthreads();
  if (threadIdx.x < 64) {
    const int c = blockIdx.x * 64 + threadIdx.x;
    if (c < d) {
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) t += red[i][threadIdx.x];
      if (accumulate) t += bf2f(out[c]);
      out[c] = f2bf(t);
    }
  }
}

template <bool RMS, bool HAS_RES>
void launch_fwd_t(int nv, dim3 grid, hipStream_t st, const bf16_t* x, const bf16_t* r,
                  const bf16_t* w, const bf16_t* b, bf16_t* s_out, bf16_t* y, float* mean,
                  float* rstd, int N, int d, float eps, uint32_t thr, float scale,
                  const int64_t* seed, int64_t site) {
#define DLTB_NF(NVV)                                                                             \
  hipLaunchKernelGGL((norm_fwd_kernel<NVV, RMS, HAS_RES>), grid, dim3(256), 0, st, x, r, w, b,   \
                     s_out, y, mean, rstd, N, d, eps, thr, scale, seed, site)
  switch (nv) {
    case 1: DLTB_NF(1); break;
    case 2: DLTB_NF(2); break;
    case 3: DLTB_NF(3); break;
    case 4: DLTB_NF(4); break;
    case 6: DLTB_NF(6); break;
    default: DLTB_NF(8); break;
  }
#undef DLTB_NF
}

int nv_for(int d) {
  int nv = cdiv(d / 8, 64);
  if (nv == 5) nv = 6;
  if (nv == 7) nv = 8;
  return nv;
}

}  // namespace

// ---------------------------------------------------------------------------------------- API
void dltb_norm_fwd(const void* x, const void* r, const void* w, const void* b, void* s_out,
                   void* y, float* mean, float* rstd, int N, int d, float eps, bool rms,
                   uint32_t thr16, float drop_scale, const int64_t* seed, int64_t site,
                   hipStream_t st) {
  const int nv = nv_for(d);
  dim3 grid(cdiv(N, kWaves));
  auto X = (const bf16_t*)x;
  auto R = (const bf16_t*)r;
  auto W = (const bf16_t*)w;
  auto B = (const bf16_t*)b;
  auto S = (bf16_t*)s_out;
  auto Y = (bf16_t*)y;
  if (rms) {
    if (r) launch_fwd_t<true, true>(nv, grid, st, X, R, W, B, S, Y, mean, rstd, N, d, eps, thr16, drop_scale, seed, site);
    else   launch_fwd_t<true, false>(nv, grid, st, X, R, W, B, S, Y, mean, rstd, N, d, eps, thr16, drop_scale, seed, site);
  } else {
    if (r) launch_fwd_t<false, true>(nv, grid, st, X, R, W, B, S, Y, mean, rstd, N, d, eps, thr16, drop_scale, seed, site);
    else   launch_fwd_t<false, false>(nv, grid, st, X, R, W, B, S, Y, mean, rstd, N, d, eps, thr16, drop_scale, seed, site);
  }
}

template <bool RMS, bool HAS_RES>
void launch_fwd_mask_t(int nv, int nb_norm, int nb_mask, hipStream_t st, const bf16_t* x, const bf16_t* r,
                       const bf16_t* w, const bf16_t* b, bf16_t* s_out, bf16_t* y, float* mean, float* rstd,
                       int N, int d, float eps, uint32_t thr, float scale, const int64_t* seed, int64_t site,
                       const MaskJob& mj) {
  const dim3 grid(nb_norm + nb_mask);
#define DLTB_NFM(NVV)                                                                                 \
  hipLaunchKernelGGL((norm_fwd_mask_kernel<NVV, RMS, HAS_RES>), grid, dim3(256), 0, st, x, r, w, b,   \
                     s_out, y, mean, rstd, N, d, eps, thr, scale, seed, site, nb_norm, mj)
  switch (nv) {
    case 1: DLTB_NFM(1); break;
    case 2: DLTB_NFM(2); break;
    case 3: DLTB_NFM(3); break;
    case 4: DLTB_NFM(4); break;
    case 6: DLTB_NFM(6); break;
    default: DLTB_NFM(8); break;
  }
#undef DLTB_NFM
}

void dltb_norm_fwd_mask(const void* x, const void* r, const void* w, const void* b, void* s_out, void* y,
                        float* mean, float* rstd, int N, int d, float eps, bool rms, uint32_t thr16,
                        float drop_scale, const int64_t* seed, int64_t site, uint32_t* mask, int B, int T,
                        int Hq, uint32_t mask_thr16, const int64_t* mask_seed, int64_t mask_site, hipStream_t st,
                        int g_begin, int g_end) {
  const int nv = nv_for(d);
  const int ng = B * Hq * (T / kMaskKeyTile) * 2;          // tile groups of the whole mask
  if (g_end < 0 || g_end > ng) g_end = ng;
  const MaskJob mj{mask, T, mask_thr16, mask_seed, mask_site, cdiv(T, 256), g_begin};
  const int nb_norm = cdiv(N, kWaves);
  const int nb_mask = g_end > g_begin ? mj.gx * (g_end - g_begin) : 0;
  auto X = (const bf16_t*)x;
  auto R = (const bf16_t*)r;
  auto W = (const bf16_t*)w;
  auto Bi = (const bf16_t*)b;
  auto S = (bf16_t*)s_out;
  auto Y = (bf16_t*)y;
  if (rms) {
    if (r) launch_fwd_mask_t<true, true>(nv, nb_norm, nb_mask, st, X, R, W, Bi, S, Y, mean, rstd, N, d, eps, thr16, drop_scale, seed, site, mj);
    else   launch_fwd_mask_t<true, false>(nv, nb_norm, nb_mask, st, X, R, W, Bi, S, Y, mean, rstd, N, d, eps, thr16, drop_scale, seed, site, mj);
  } else {
    if (r) launch_fwd_mask_t<false, true>(nv, nb_norm, nb_mask, st, X, R, W, Bi, S, Y, mean, rstd, N, d, eps, thr16, drop_scale, seed, site, mj);
    else   launch_fwd_mask_t<false, false>(nv, nb_norm, nb_mask, st, X, R, W, Bi, S, Y, mean, rstd, N, d, eps, thr16, drop_scale, seed, site, mj);
  }
}

int dltb_norm_bwd_partials(int N) {
  int P = N / 32;
  if (P < 1) P = 1;
  if (P > 128) P = 128;
  return P;
}

void dltb_norm_bwd_dx(const void* dy, const void* s, const void* w, const float* mean,
                      const float* rstd, const void* dres, void* dx, int N, int d, bool rms,
                      hipStream_t st) {
  const int nv = nv_for(d);
  auto DY = (const bf16_t*)dy;
  auto S = (const bf16_t*)s;
  auto W = (const bf16_t*)w;
  auto DR = (const bf16_t*)dres;
  auto DX = (bf16_t*)dx;
  dim3 grid(cdiv(N, kWaves));
#define DLTB_NB(NVV, RMSV, RESV)                                                                 \
  hipLaunchKernelGGL((norm_bwd_dx_kernel<NVV, RMSV, RESV>), grid, dim3(256), 0, st, DY, S, W,    \
                     mean, rstd, DR, DX, N, d)
#define DLTB_NB_NV(RMSV, RESV)            \
  switch (nv) {                           \
    case 1: DLTB_NB(1, RMSV, RESV); break; \
    case 2: DLTB_NB(2, RMSV, RESV); break; \
    case 3: DLTB_NB(3, RMSV, RESV); break; \
    case 4: DLTB_NB(4, RMSV, RESV); break; \
    case 6: DLTB_NB(6, RMSV, RESV); break; \
    default: DLTB_NB(8, RMSV, RESV); break; \
  }
  if (rms) {
    if (dres) { DLTB_NB_NV(true, true) } else { DLTB_NB_NV(true, false) }
  } else {
    if (dres) { DLTB_NB_NV(false, true) } else { DLTB_NB_NV(false, false) }
  }
#undef DLTB_NB_NV
#undef DLTB_NB
}

void dltb_norm_bwd_dgamma(const void* dy, const void* s, const float* mean, const float* rstd,
                          float* part, void* gw, void* gb, int accumulate, int N, int d, bool rms,
                          hipStream_t st) {
  auto DY = (const bf16_t*)dy;
  auto S = (const bf16_t*)s;
  const int P = dltb_norm_bwd_partials(N);
  const int rps = cdiv(N, P);
  dim3 g2(cdiv(d, 512), P);
  if (rms)
    hipLaunchKernelGGL(norm_dgamma_kernel<true>, g2, dim3(256), 0, st, DY, S, mean, rstd, part, N, d, rps);
  else
    hipLaunchKernelGGL(norm_dgamma_kernel<false>, g2, dim3(256), 0, st, DY, S, mean, rstd, part, N, d, rps);
  hipLaunchKernelGGL(norm_colreduce_kernel, dim3(cdiv(d, 64), rms ? 1 : 2), dim3(256), 0, st, part, P, d,
                     (bf16_t*)gw, rms ? nullptr : (bf16_t*)gb, accumulate);
}

// ---- fused backward (dx + column partials); rows per wave chosen for >= 256 workgroups
static int dltb_norm_bwd_fused_rpw(int N) {
  int rpw = N / (kFusedWaves * 256);
  return rpw < 1 ? 1 : rpw;
}

int dltb_norm_bwd_fused_blocks(int N) { return cdiv(N, kFusedWaves * dltb_norm_bwd_fused_rpw(N)); }

bool dltb_norm_bwd_fused_supported(int d) { return d % 8 == 0 && nv_for(d) <= 4; }

namespace {
struct FusedDrop {
  bf16_t* dm;
  uint32_t thr16;
  float scale;
  const int64_t* seed;
  int64_t site;
};
template <int NV, bool RMS, bool RES, int XS>
void launch_bwd_fused(int N, int d, hipStream_t st, const bf16_t* dy, const bf16_t* s, const bf16_t* w,
                      const float* mean, const float* rstd, const bf16_t* dres, bf16_t* dx, float* part,
                      const FusedDrop& fd) {
  const int rpw = dltb_norm_bwd_fused_rpw(N);
  constexpr int K = (RMS ? 1 : 2) + (XS ? 1 : 0);
  const size_t one = (size_t)K * kFusedWaves * d * sizeof(float);
  const bool one_fold = one <= kFoldLdsMax;
  if (one_fold && one > 65536) {
    static bool attr = false;                 // per instantiation: allow the large dynamic LDS image
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)norm_bwd_fused_kernel<NV, RMS, RES, XS>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kFoldLdsMax);
      attr = true;
    }
  }
  hipLaunchKernelGGL((norm_bwd_fused_kernel<NV, RMS, RES, XS>), dim3(dltb_norm_bwd_fused_blocks(N)),
                     dim3(kFusedWaves * 64), one_fold ? one : (size_t)kFusedWaves * d * sizeof(float), st, dy, s, w,
                     mean, rstd, dres, dx, part, N, d, rpw, fd.dm, fd.thr16, fd.scale, fd.seed, fd.site, one_fold);
}
template <int NV, bool RMS, bool RES>
void launch_bwd_fused_xs(int xs, int N, int d, hipStream_t st, const bf16_t* dy, const bf16_t* s,
                         const bf16_t* w, const float* mean, const float* rstd, const bf16_t* dres,
                         bf16_t* dx, float* part, const FusedDrop& fd) {
  if (xs == 2) launch_bwd_fused<NV, RMS, RES, 2>(N, d, st, dy, s, w, mean, rstd, dres, dx, part, fd);
  else if (xs == 1) launch_bwd_fused<NV, RMS, RES, 1>(N, d, st, dy, s, w, mean, rstd, dres, dx, part, fd);
  else launch_bwd_fused<NV, RMS, RES, 0>(N, d, st, dy, s, w, mean, rstd, dres, dx, part, fd);
}
template <int NV, bool RMS>
void launch_bwd_fused_nv(bool res, int xs, int N, int d, hipStream_t st, const bf16_t* dy,
                         const bf16_t* s, const bf16_t* w, const float* mean, const float* rstd,
                         const bf16_t* dres, bf16_t* dx, float* part, const FusedDrop& fd) {
  if (res) launch_bwd_fused_xs<NV, RMS, true>(xs, N, d, st, dy, s, w, mean, rstd, dres, dx, part, fd);
  else launch_bwd_fused_xs<NV, RMS, false>(xs, N, d, st, dy, s, w, mean, rstd, dres, dx, part, fd);
}
}  // namespace

bool dltb_norm_bwd_fused(const void* dy, const void* s, const void* w, const float* mean,
                         const float* rstd, const void* dres, void* dx, float* part, int N, int d,
                         bool rms, bool dxsum, hipStream_t st, void* dm, uint32_t thr16, float drop_scale,
                         const int64_t* seed, int64_t site) {
  if (!dltb_norm_bwd_fused_supported(d)) return false;
  auto DY = (const bf16_t*)dy;
  auto S = (const bf16_t*)s;
  auto W = (const bf16_t*)w;
  auto DR = (const bf16_t*)dres;
  auto DX = (bf16_t*)dx;
  const bool res = dres != nullptr;
  const int xs = dm != nullptr ? 2 : (dxsum ? 1 : 0);
  const FusedDrop fd{(bf16_t*)dm, thr16, drop_scale, seed, site};
#define DLTB_NBF(NVV)                                                                                    \
  do {                                                                                                   \
    if (rms) launch_bwd_fused_nv<NVV, true>(res, xs, N, d, st, DY, S, W, mean, rstd, DR, DX, part, fd);  \
    else launch_bwd_fused_nv<NVV, false>(res, xs, N, d, st, DY, S, W, mean, rstd, DR, DX, part, fd);     \
  } while (0)
  switch (nv_for(d)) {
    case 1: DLTB_NBF(1); break;
    case 2: DLTB_NBF(2); break;
    case 3: DLTB_NBF(3); break;
    default: DLTB_NBF(4); break;
  }
#undef DLTB_NBF
  return true;
}

void dltb_norm_bwd(const void* dy, const void* s, const void* w, const float* mean,
                   const float* rstd, const void* dres, void* dx, float* part, void* gw, void* gb,
                   int accumulate, int N, int d, bool rms, hipStream_t st) {
  dltb_norm_bwd_dx(dy, s, w, mean, rstd, dres, dx, N, d, rms, st);
  dltb_norm_bwd_dgamma(dy, s, mean, rstd, part, gw, gb, accumulate, N, d, rms, st);
}
