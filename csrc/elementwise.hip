// Memory-bound elementwise kernels for gfx950 (all bf16 I/O as 16-byte vectors, fp32 math).
//
//   gelu_fwd            g = gelu_erf(f)                                   (nn.GELU, train_harness.py:120)
//   gelu_bwd_colsum     df = dg * gelu'(f), plus fp32 column partials of df (-> fc1 bias grad)
//   colsum              fp32 column partials of a [N, k] bf16 matrix      (bias grads)
//   colreduce           sum partial rows -> bf16 gradient slot (overwrite / accumulate)
//   dropout_add         out = x + dropout(r)                              (residual + Dropout)
//   dropout_bwd         out = dropout_mask(g) * 1/(1-p)                   (mask regenerated)
//   swiglu_fwd/bwd      h = silu(gate) * up                               (Mistral-shape FFN)
//   rope_fwd/bwd        rotate-half RoPE in place on the q/k columns of a fused qkv buffer
//   f32_from_bf16       dst (+)= float(src)
//   transpose           dst[C, R] = src[R, C]^T (64x64 LDS tiles; cached W^T for dgrad GEMMs)
#include "common.h"
#include "launchers.h"

namespace {

// ------------------------------------------------------------------------------------ GELU
DLTB_DEV float gelu_f(float x) { return gelu_fwd_f(x); }
DLTB_DEV float gelu_grad(float x) { return gelu_grad_f(x); }

__global__ __launch_bounds__(256) void gelu_fwd_kernel(const bf16_t* __restrict__ f,
                                                      bf16_t* __restrict__ g, long n8) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float v[8];
    unpack8(ld16<uint4>(f + i * 8), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = gelu_f(v[e]);
    *reinterpret_cast<uint4*>(g + i * 8) = pack8(v);
  }
}

// g = GELU(f) and gp = GELU'(f) in one pass (the erf and exp of the derivative are the forward's own): the
// backward's dGELU then rides in the fc2 data-gradient GEMM's epilogue (gemm_rs aux) and f is not kept.
__global__ __launch_bounds__(256) void gelu_fwd_grad_kernel(const bf16_t* __restrict__ f, bf16_t* __restrict__ g,
                                                           bf16_t* __restrict__ gp, long n8) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float v[8], d[8];
    unpack8(ld16<uint4>(f + i * 8), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float ex;                                          // exp(-x^2 / 2)
      const float x = v[e];
      const float cdf = 0.5f * (1.f + erf_fast(x * 0.70710678118654752f, &ex));
      v[e] = x * cdf;
      d[e] = cdf + x * 0.39894228040143268f * ex;
    }
    *reinterpret_cast<uint4*>(g + i * 8) = pack8(v);
    *reinterpret_cast<uint4*>(gp + i * 8) = pack8(d);
  }
}

// Column-partials layout shared by gelu_bwd_colsum and colsum:
//   block (bx, by): columns [bx*512, bx*512+512), rows [by*rps, (by+1)*rps)
//   thread: lane = tid & 63 -> 8 columns, phase = tid >> 6 -> every 4th row
//   out: part[by][k]
template <bool GELU>
__global__ __launch_bounds__(256) void colsum_kernel(const bf16_t* __restrict__ src,
                                                    const bf16_t* __restrict__ f,
                                                    bf16_t* __restrict__ dst, float* __restrict__ part,
                                                    int N, int k, int rps) {
  __shared__ __attribute__((aligned(16))) float red[4][512];
  const int lane = threadIdx.x & 63, phase = threadIdx.x >> 6;
  const int col = blockIdx.x * 512 + lane * 8;
  const int r0 = blockIdx.y * rps;
  const int r1 = min(N, r0 + rps);
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  if (col < k) {
    for (int r = r0 + phase; r < r1; r += 4) {
      const size_t off = (size_t)r * k + col;
      float v[8];
      unpack8(ld16<uint4>(src + off), v);
      if (GELU) {
        float fv[8];
        unpack8(ld16<uint4>(f + off), fv);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] *= gelu_grad(fv[e]);
        uint4 o = pack8(v);
        *reinterpret_cast<uint4*>(dst + off) = o;
        unpack8(o, v);   // bias grad of the rounded df, as a separate reduction would see it
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[phase][lane * 8 + e] = acc[e];
  __syncthreads();
  for (int c = threadIdx.x; c < 512; c += 256) {
    const int gc = blockIdx.x * 512 + c;
    if (gc < k) part[(size_t)blockIdx.y * k + gc] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
  }
}

// sum P partial rows of [P][k] -> bf16 out (overwrite / accumulate); 16 column quads x 16 row
// phases per 256-thread block, float4 loads.
__global__ __launch_bounds__(256) void colreduce_kernel(const float* __restrict__ part, int P,
                                                       int k, bf16_t* __restrict__ out,
                                                       int accumulate) {
  __shared__ float red[16][65];
  const int cq = threadIdx.x & 15, ph = threadIdx.x >> 4;
  const int c0 = blockIdx.x * 64 + cq * 4;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c0 < k) {
    for (int p = ph; p < P; p += 16) {
      const float4 v = *reinterpret_cast<const float4*>(part + (size_t)p * k + c0);
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
    if (c < k) {
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) t += red[i][threadIdx.x];
      if (accumulate) t += bf2f(out[c]);
      out[c] = f2bf(t);
    }
  }
}

// ------------------------------------------------------------------------------- dropout
template <bool ADD>
__global__ __launch_bounds__(256) void dropout_kernel(const bf16_t* __restrict__ x,
                                                     const bf16_t* __restrict__ r,
                                                     bf16_t* __restrict__ out, long n8, int cols,
                                                     uint32_t thr16, float scale,
                                                     const int64_t* __restrict__ seed_ptr,
                                                     int64_t site) {
  const uint64_t seed = thr16 ? site_seed(seed_ptr, site) : 0ull;
  const int cv = cols >> 3;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const uint32_t row = (uint32_t)(i / cv);
    const uint32_t col0 = (uint32_t)(i - (long)row * cv) * 8;
    float rv[8];
    unpack8(ld16<uint4>(r + i * 8), rv);
    if (thr16) {
      const uint32_t rk = rng_row_key(seed, row);
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        const uint32_t h = rng_pair(rk, rng_col_key(seed, col0 + e));
        rv[e] = keep_lo(h, thr16) ? rv[e] * scale : 0.f;
        rv[e + 1] = keep_hi(h, thr16) ? rv[e + 1] * scale : 0.f;
      }
    }
    if (ADD) {
      float xv[8];
      unpack8(ld16<uint4>(x + i * 8), xv);
#pragma unroll
      for (int e = 0; e < 8; ++e) rv[e] += xv[e];
    }
    *reinterpret_cast<uint4*>(out + i * 8) = pack8(rv);
  }
}

// ------------------------------------------------------------------------------- SwiGLU
DLTB_DEV float sigmoid_f(float x) { return 1.f / (1.f + __expf(-x)); }

// gu: [N, 2F] = [gate | up]; h: [N, F]
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const bf16_t* __restrict__ gu,
                                                        bf16_t* __restrict__ h, int N, int F) {
  const long n8 = (long)N * F / 8;
  const int fv = F >> 3;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const long row = i / fv;
    const long c = (i - row * fv) * 8;
    float g[8], u[8], o[8];
    unpack8(ld16<uint4>(gu + row * 2 * F + c), g);
    unpack8(ld16<uint4>(gu + row * 2 * F + F + c), u);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = g[e] * sigmoid_f(g[e]) * u[e];
    *reinterpret_cast<uint4*>(h + row * F + c) = pack8(o);
  }
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const bf16_t* __restrict__ dh,
                                                        const bf16_t* __restrict__ gu,
                                                        bf16_t* __restrict__ dgu, int N, int F) {
  const long n8 = (long)N * F / 8;
  const int fv = F >> 3;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const long row = i / fv;
    const long c = (i - row * fv) * 8;
    float g[8], u[8], d[8], dg[8], du[8];
    unpack8(ld16<uint4>(gu + row * 2 * F + c), g);
    unpack8(ld16<uint4>(gu + row * 2 * F + F + c), u);
    unpack8(ld16<uint4>(dh + row * F + c), d);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float s = sigmoid_f(g[e]);
      const float silu = g[e] * s;
      du[e] = d[e] * silu;
      dg[e] = d[e] * u[e] * s * (1.f + g[e] * (1.f - s));
    }
    *reinterpret_cast<uint4*>(dgu + row * 2 * F + c) = pack8(dg);
    *reinterpret_cast<uint4*>(dgu + row * 2 * F + F + c) = pack8(du);
  }
}

// ------------------------------------------------------------------------------- RoPE
// qkv rows of width `stride`; q heads [0, Hq*D), k heads [Hq*D, (Hq+Hkv)*D).  cos/sin: [T, D/2]
// fp32 host-built tables.  Each thread rotates 8 consecutive pairs (i, i + D/2) of one head.
template <bool INV>
__global__ __launch_bounds__(256) void rope_kernel(bf16_t* __restrict__ qkv,
                                                  const float* __restrict__ cosb,
                                                  const float* __restrict__ sinb, int N, int T,
                                                  int heads, int D, int stride) {
  const int half = D >> 1;
  const int hv = half >> 3;                       // 8-pair groups per head
  const long total = (long)N * heads * hv;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long row = i / (heads * hv);
    const int rem = (int)(i - row * heads * hv);
    const int h = rem / hv;
    const int p0 = (rem - h * hv) * 8;
    const int t = (int)(row % T);
    bf16_t* base = qkv + row * stride + (long)h * D;
    float x1[8], x2[8], o1[8], o2[8];
    unpack8(ld16<uint4>(base + p0), x1);
    unpack8(ld16<uint4>(base + half + p0), x2);
    const float* cr = cosb + (long)t * half + p0;
    const float* sr = sinb + (long)t * half + p0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float c = cr[e];
      const float s = INV ? -sr[e] : sr[e];
      o1[e] = x1[e] * c - x2[e] * s;
      o2[e] = x2[e] * c + x1[e] * s;
    }
    *reinterpret_cast<uint4*>(base + p0) = pack8(o1);
    *reinterpret_cast<uint4*>(base + half + p0) = pack8(o2);
  }
}

// ------------------------------------------------------------------------------- casts
__global__ __launch_bounds__(256) void f32_from_bf16_kernel(float* __restrict__ dst,
                                                           const bf16_t* __restrict__ src, long n8,
                                                           int accumulate) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float v[8];
    unpack8(ld16<uint4>(src + i * 8), v);
    float4* d = reinterpret_cast<float4*>(dst + i * 8);
    if (accumulate) {
      float4 a = d[0], b = d[1];
      d[0] = make_float4(a.x + v[0], a.y + v[1], a.z + v[2], a.w + v[3]);
      d[1] = make_float4(b.x + v[4], b.y + v[5], b.z + v[6], b.w + v[7]);
    } else {
      d[0] = make_float4(v[0], v[1], v[2], v[3]);
      d[1] = make_float4(v[4], v[5], v[6], v[7]);
    }
  }
}

int ew_grid(long n8) {
  long g = (n8 + 255) / 256;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

int colsum_splits(int N) {
  int s = N / 32;
  if (s < 1) s = 1;
  if (s > 128) s = 128;
  return s;
}

// ----------------------------------------------------------------------------- transpose
// 64x64 tile through LDS (+1 column pad: conflict-free column reads); 256 threads, each moves
// 16 elements; rows read and written as 8-byte (4 x bf16) vectors along the contiguous dim.
__global__ __launch_bounds__(256) void transpose_kernel(const bf16_t* __restrict__ src,
                                                       bf16_t* __restrict__ dst, int R, int C,
                                                       long sbs, long dbs) {
  __shared__ bf16_t tile[64][65];
  src += blockIdx.z * sbs;                                     // batch: equally spaced matrices
  dst += blockIdx.z * dbs;
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;     // 16 x 16 threads, 4 columns each
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int r = r0 + ty + 16 * k, c = c0 + tx * 4;
    if (r < R && c < C) {
      const uint2 v = *reinterpret_cast<const uint2*>(src + (size_t)r * C + c);
      tile[ty + 16 * k][tx * 4 + 0] = (bf16_t)(v.x & 0xFFFF);
      tile[ty + 16 * k][tx * 4 + 1] = (bf16_t)(v.x >> 16);
      tile[ty + 16 * k][tx * 4 + 2] = (bf16_t)(v.y & 0xFFFF);
      tile[ty + 16 * k][tx * 4 + 3] = (bf16_t)(v.y >> 16);
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = c0 + ty + 16 * k, r = r0 + tx * 4;          // output row c, columns r .. r+3
    if (c < C && r < R) {
      uint2 v;
      v.x = (uint32_t)tile[tx * 4 + 0][ty + 16 * k] | ((uint32_t)tile[tx * 4 + 1][ty + 16 * k] << 16);
      v.y = (uint32_t)tile[tx * 4 + 2][ty + 16 * k] | ((uint32_t)tile[tx * 4 + 3][ty + 16 * k] << 16);
      *reinterpret_cast<uint2*>(dst + (size_t)c * R + r) = v;
    }
  }
}

// y = x * (num[0] / den[0]) with the scale read on the device (no host sync); block 0 thread 0
// also stores the scale to g_out (re-used by the next kernel, e.g. as a GEMM alpha).
__global__ __launch_bounds__(256) void scale_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                   long n8, const float* __restrict__ num,
                                                   const float* __restrict__ den, float* __restrict__ g_out) {
  const float s = num[0] / (den ? den[0] : 1.f);
  if (g_out && blockIdx.x == 0 && threadIdx.x == 0) g_out[0] = s;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float f[8];
    unpack8(ld16<uint4>(x + i * 8), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] *= s;
    *reinterpret_cast<uint4*>(y + i * 8) = pack8(f);
  }
}

}  // namespace

void dltb_scale(const void* x, void* y, long n, const float* num, const float* den, float* g_out,
                hipStream_t st) {
  const long n8 = n / 8;
  long grid = (n8 + 255) / 256;
  if (grid > 2048) grid = 2048;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(scale_kernel, dim3(grid), dim3(256), 0, st, (const bf16_t*)x, (bf16_t*)y, n8, num,
                     den, g_out);
}

// ---------------------------------------------------------------------------------------- API
void dltb_gelu_fwd(const void* f, void* g, long n, hipStream_t st) {
  const long n8 = n / 8;
  hipLaunchKernelGGL(gelu_fwd_kernel, dim3(ew_grid(n8)), dim3(256), 0, st, (const bf16_t*)f,
                     (bf16_t*)g, n8);
}

void dltb_gelu_fwd_grad(const void* f, void* g, void* gp, long n, hipStream_t st) {
  const long n8 = n / 8;
  hipLaunchKernelGGL(gelu_fwd_grad_kernel, dim3(ew_grid(n8)), dim3(256), 0, st, (const bf16_t*)f, (bf16_t*)g,
                     (bf16_t*)gp, n8);
}

int dltb_colsum_partials(int N) { return colsum_splits(N); }

// dg -> df (written), bias grad -> db slot; `part` must hold colsum_partials(N) * k floats
void dltb_gelu_bwd(const void* dg, const void* f, void* df, float* part, void* db, int accumulate,
                   int N, int k, hipStream_t st) {
  const int P = colsum_splits(N);
  const int rps = cdiv(N, P);
  dim3 grid(cdiv(k, 512), P);
  hipLaunchKernelGGL(colsum_kernel<true>, grid, dim3(256), 0, st, (const bf16_t*)dg,
                     (const bf16_t*)f, (bf16_t*)df, part, N, k, rps);
  if (db)
    hipLaunchKernelGGL(colreduce_kernel, dim3(cdiv(k, 64)), dim3(256), 0, st, part, P, k,
                       (bf16_t*)db, accumulate);
}

void dltb_colsum(const void* src, float* part, void* out, int accumulate, int N, int k,
                 hipStream_t st) {
  const int P = colsum_splits(N);
  const int rps = cdiv(N, P);
  dim3 grid(cdiv(k, 512), P);
  hipLaunchKernelGGL(colsum_kernel<false>, grid, dim3(256), 0, st, (const bf16_t*)src, nullptr,
                     nullptr, part, N, k, rps);
  hipLaunchKernelGGL(colreduce_kernel, dim3(cdiv(k, 64)), dim3(256), 0, st, part, P, k,
                     (bf16_t*)out, accumulate);
}

void dltb_dropout(const void* x, const void* r, void* out, long n, int cols, uint32_t thr16,
                  float scale, const int64_t* seed, int64_t site, hipStream_t st) {
  const long n8 = n / 8;
  if (x)
    hipLaunchKernelGGL(dropout_kernel<true>, dim3(ew_grid(n8)), dim3(256), 0, st,
                       (const bf16_t*)x, (const bf16_t*)r, (bf16_t*)out, n8, cols, thr16, scale,
                       seed, site);
  else
    hipLaunchKernelGGL(dropout_kernel<false>, dim3(ew_grid(n8)), dim3(256), 0, st, nullptr,
                       (const bf16_t*)r, (bf16_t*)out, n8, cols, thr16, scale, seed, site);
}

void dltb_swiglu_fwd(const void* gu, void* h, int N, int F, hipStream_t st) {
  hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(ew_grid((long)N * F / 8)), dim3(256), 0, st,
                     (const bf16_t*)gu, (bf16_t*)h, N, F);
}

void dltb_swiglu_bwd(const void* dh, const void* gu, void* dgu, int N, int F, hipStream_t st) {
  hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(ew_grid((long)N * F / 8)), dim3(256), 0, st,
                     (const bf16_t*)dh, (const bf16_t*)gu, (bf16_t*)dgu, N, F);
}

void dltb_rope(void* qkv, const float* cosb, const float* sinb, int N, int T, int heads, int D,
               int stride, bool inverse, hipStream_t st) {
  const long total = (long)N * heads * (D / 16);
  if (inverse)
    hipLaunchKernelGGL(rope_kernel<true>, dim3(ew_grid(total)), dim3(256), 0, st, (bf16_t*)qkv,
                       cosb, sinb, N, T, heads, D, stride);
  else
    hipLaunchKernelGGL(rope_kernel<false>, dim3(ew_grid(total)), dim3(256), 0, st, (bf16_t*)qkv,
                       cosb, sinb, N, T, heads, D, stride);
}

void dltb_f32_from_bf16(float* dst, const void* src, long n, int accumulate, hipStream_t st) {
  const long n8 = n / 8;
  hipLaunchKernelGGL(f32_from_bf16_kernel, dim3(ew_grid(n8)), dim3(256), 0, st, dst,
                     (const bf16_t*)src, n8, accumulate);
}

void dltb_transpose(const void* src, void* dst, int R, int C, hipStream_t st) {
  dltb_transpose_batched(src, dst, R, C, 1, 0, 0, st);
}

void dltb_transpose_batched(const void* src, void* dst, int R, int C, int nb, long sbs, long dbs,
                            hipStream_t st) {
  hipLaunchKernelGGL(transpose_kernel, dim3(cdiv(C, 64), cdiv(R, 64), nb), dim3(256), 0, st,
                     (const bf16_t*)src, (bf16_t*)dst, R, C, sbs, dbs);
}
