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
#include "common.h"

namespace {

constexpr int kRowsPerWave = 4;   // backward: rows per wave
constexpr int kWaves = 4;

template <int NV, bool RMS, bool HAS_RES>
__global__ __launch_bounds__(256) void norm_fwd_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ r, const bf16_t* __restrict__ w,
    const bf16_t* __restrict__ b, bf16_t* __restrict__ s_out, bf16_t* __restrict__ y,
    float* __restrict__ mean_out, float* __restrict__ rstd_out, int N, int d, float eps,
    uint32_t thr16, float drop_scale, const int64_t* __restrict__ seed_ptr, int64_t site) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kWaves + (threadIdx.x >> 6);
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
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int idx = j * 64 + lane;
    if (idx < nvec) {
      uint4 xv = ld16<uint4>(x + base + idx * 8);
      unpack8(xv, v[j]);
      if (HAS_RES) {
        float rv[8];
        uint4 rr = ld16<uint4>(r + base + idx * 8);
        unpack8(rr, rv);
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
      unpack8(ld16<uint4>(w + idx * 8), wv);
      if (!RMS) {
        float bv[8];
        unpack8(ld16<uint4>(b + idx * 8), bv);
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

// dgamma/dbeta partials: part[blk][0][d] (dgamma), part[blk][1][d] (dbeta)
template <int NV, bool RMS, bool HAS_RES_GRAD>
__global__ __launch_bounds__(256) void norm_bwd_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ s, const bf16_t* __restrict__ w,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    const bf16_t* __restrict__ dres, bf16_t* __restrict__ dx, float* __restrict__ part, int N,
    int d) {
  extern __shared__ __attribute__((aligned(16))) float lds[];   // [2][d]
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int nvec = d >> 3;
  for (int i = threadIdx.x; i < 2 * d; i += blockDim.x) lds[i] = 0.f;
  __syncthreads();
  float gacc[NV][8], bacc[NV][8];
#pragma unroll
  for (int j = 0; j < NV; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) { gacc[j][e] = 0.f; bacc[j][e] = 0.f; }
  const int row0 = (blockIdx.x * kWaves + wid) * kRowsPerWave;
  for (int rr = 0; rr < kRowsPerWave; ++rr) {
    const int row = row0 + rr;
    if (row >= N) break;
    const size_t base = (size_t)row * d;
    const float mean = RMS ? 0.f : mean_in[row];
    const float rstd = rstd_in[row];
    float s1 = 0.f, s2 = 0.f;   // sum(w*dy), sum(w*dy*xhat)
    // pass 1: row statistics + dgamma/dbeta partials
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
          const float xh = (xv[e] - mean) * rstd;
          const float g = dyv[e] * wv[e];
          s1 += g;
          s2 += g * xh;
          gacc[j][e] += dyv[e] * xh;
          bacc[j][e] += dyv[e];
        }
      }
    }
    s1 = RMS ? 0.f : wave_sum(s1) / (float)d;
    s2 = wave_sum(s2) / (float)d;
    // pass 2: dx (re-reads hit L1/L2)
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int idx = j * 64 + lane;
      if (idx < nvec) {
        float dyv[8], xv[8], wv[8], o[8];
        unpack8(ld16<uint4>(dy + base + idx * 8), dyv);
        unpack8(ld16<uint4>(s + base + idx * 8), xv);
        unpack8(ld16<uint4>(w + idx * 8), wv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float xh = (xv[e] - mean) * rstd;
          o[e] = rstd * (dyv[e] * wv[e] - s1 - xh * s2);
        }
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
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int idx = j * 64 + lane;
    if (idx < nvec) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        atomicAdd(&lds[idx * 8 + e], gacc[j][e]);
        if (!RMS) atomicAdd(&lds[d + idx * 8 + e], bacc[j][e]);
      }
    }
  }
  __syncthreads();
  float* out = part + (size_t)blockIdx.x * 2 * d;
  for (int i = threadIdx.x; i < 2 * d; i += blockDim.x) out[i] = lds[i];
}

// sum P partial rows of [P][2][d] -> bf16 gamma grad (and beta grad if gb != null)
__global__ __launch_bounds__(256) void norm_colreduce_kernel(const float* __restrict__ part, int P,
                                                             int d, bf16_t* __restrict__ gw,
                                                             bf16_t* __restrict__ gb,
                                                             int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= d) return;
  float a = 0.f, bsum = 0.f;
  for (int p = 0; p < P; ++p) {
    a += part[(size_t)p * 2 * d + c];
    if (gb) bsum += part[(size_t)p * 2 * d + d + c];
  }
  if (accumulate) {
    a += bf2f(gw[c]);
    if (gb) bsum += bf2f(gb[c]);
  }
  gw[c] = f2bf(a);
  if (gb) gb[c] = f2bf(bsum);
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

int dltb_norm_bwd_partials(int N) { return cdiv(N, kWaves * kRowsPerWave); }

void dltb_norm_bwd(const void* dy, const void* s, const void* w, const float* mean,
                   const float* rstd, const void* dres, void* dx, float* part, void* gw, void* gb,
                   int accumulate, int N, int d, bool rms, hipStream_t st) {
  const int nv = nv_for(d);
  const int P = dltb_norm_bwd_partials(N);
  dim3 grid(P);
  size_t lds = (size_t)2 * d * sizeof(float);
  auto DY = (const bf16_t*)dy;
  auto S = (const bf16_t*)s;
  auto W = (const bf16_t*)w;
  auto DR = (const bf16_t*)dres;
  auto DX = (bf16_t*)dx;
#define DLTB_NB(NVV, RMSV, RESV)                                                                 \
  hipLaunchKernelGGL((norm_bwd_kernel<NVV, RMSV, RESV>), grid, dim3(256), lds, st, DY, S, W,     \
                     mean, rstd, DR, DX, part, N, d)
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
  hipLaunchKernelGGL(norm_colreduce_kernel, dim3(cdiv(d, 256)), dim3(256), 0, st, part, P, d,
                     (bf16_t*)gw, rms ? nullptr : (bf16_t*)gb, accumulate);
}
