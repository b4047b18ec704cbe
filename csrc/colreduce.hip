// Batched column reductions for the backward pass (bias and norm-weight gradients).
//
// A transformer block's backward needs eight column sums (the biases of the four linears, the
// LayerNorm gamma/beta pairs).  Instead of two launches per sum (partials + reduce), the block
// issues:
//   colpart  - ONE launch per producer site computing fp32 column partials of up to 3 matrices
//              (blockIdx.z = segment), fused with the elementwise work that produces them:
//                PLAIN  part0 = sum_r a
//                GELU   dst = a * gelu'(b)              part0 = sum_r dst   (fc1 bias)
//                DROP   dst = dropout_mask(a) / (1-p)   part0 = sum_r dst   (fc2 bias)
//                LN     part0 = sum_r a * (b - mean) * rstd,  part1 = sum_r a  (gamma, beta)
//                RMS    part0 = sum_r a * b * rstd
//   colreduce_multi - ONE launch at the end of the block summing every partial set into its
//              bf16 gradient slot (overwrite or accumulate), blockIdx.y = segment.
// Partials layout: part[o][P][k], block (bx, by): columns [bx*512, +512), rows [by*rps, +rps),
// lane -> 8 columns, 4 waves -> every 4th row, folded through LDS.
#include "common.h"
#include "launchers.h"

namespace {

DLTB_DEV float gelu_grad_c(float x) { return gelu_grad_f(x); }

struct ColPartArgs {
  DltbColPartSeg seg[3];
  int P;
  uint32_t thr16;
  float drop_scale;
  const int64_t* seed_ptr;
};

__global__ __launch_bounds__(256) void colpart_kernel(ColPartArgs A) {
  __shared__ __attribute__((aligned(16))) float red[2][4][512];
  const DltbColPartSeg& S = A.seg[blockIdx.z];
  const int lane = threadIdx.x & 63, phase = threadIdx.x >> 6;
  const int k = S.k;
  if ((int)blockIdx.x * 512 >= k) return;             // block-uniform: this segment is narrower
  const int col = blockIdx.x * 512 + lane * 8;
  const int rps = (S.N + A.P - 1) / A.P;
  const int r0 = blockIdx.y * rps;
  const int r1 = min(S.N, r0 + rps);
  const int kind = S.kind;
  DLTB_DCHECK(k % 8 == 0 && kind >= 0 && kind <= 4 && r1 <= S.N);
  float a0[8], a1[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { a0[e] = 0.f; a1[e] = 0.f; }
  uint64_t seed = 0;
  if (kind == DLTB_COLPART_DROP && A.thr16) seed = site_seed(A.seed_ptr, S.site);
  if (col < k) {
    for (int r = r0 + phase; r < r1; r += 4) {
      const size_t off = (size_t)r * k + col;
      float v[8];
      unpack8(ld16<uint4>(S.a + off), v);
      if (kind == DLTB_COLPART_GELU) {
        float fv[8];
        unpack8(ld16<uint4>(S.b + off), fv);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] *= gelu_grad_c(fv[e]);
        const uint4 o = pack8(v);
        *reinterpret_cast<uint4*>(S.dst + off) = o;
        unpack8(o, v);                                   // sum the rounded value the GEMM consumes
      } else if (kind == DLTB_COLPART_DROP) {
        if (A.thr16) {
          const uint32_t rk = rng_row_key(seed, (uint32_t)r);
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            const uint32_t h = rng_pair(rk, rng_col_key(seed, (uint32_t)(col + e)));
            v[e] = keep_lo(h, A.thr16) ? v[e] * A.drop_scale : 0.f;
            v[e + 1] = keep_hi(h, A.thr16) ? v[e + 1] * A.drop_scale : 0.f;
          }
        }
        const uint4 o = pack8(v);
        *reinterpret_cast<uint4*>(S.dst + off) = o;
        unpack8(o, v);
      } else if (kind == DLTB_COLPART_LN || kind == DLTB_COLPART_RMS) {
        float xv[8];
        unpack8(ld16<uint4>(S.b + off), xv);
        const float mean = kind == DLTB_COLPART_LN ? S.mean[r] : 0.f;
        const float rstd = S.rstd[r];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          a1[e] += v[e];
          v[e] *= (xv[e] - mean) * rstd;
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) a0[e] += v[e];
    }
  }
  const bool two = kind == DLTB_COLPART_LN;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[0][phase][lane * 8 + e] = a0[e];
    if (two) red[1][phase][lane * 8 + e] = a1[e];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 512; c += 256) {
    const int gc = blockIdx.x * 512 + c;
    if (gc < k) {
      S.part[(size_t)blockIdx.y * k + gc] = red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c];
      if (two)
        S.part[(size_t)(A.P + blockIdx.y) * k + gc] = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
    }
  }
}

struct ColRedArgs {
  DltbColRedSeg seg[DLTB_COLRED_MAX];
};

// 16 column quads x 16 row phases per block, float4 loads; blockIdx.y = segment
__global__ __launch_bounds__(256) void colreduce_multi_kernel(ColRedArgs A) {
  __shared__ float red[16][65];
  const DltbColRedSeg& S = A.seg[blockIdx.y];
  const int k = S.k;
  if ((int)blockIdx.x * 64 >= k) return;
  const int cq = threadIdx.x & 15, ph = threadIdx.x >> 4;
  const int c0 = blockIdx.x * 64 + cq * 4;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c0 < k) {
    // four partial rows in flight per lane (independent sums, added in a fixed order)
    float4 b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) b[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    int p = ph;
    for (; p + 48 < S.P; p += 64) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(S.part + (size_t)(p + 16 * u) * k + c0);
#pragma unroll
      for (int u = 0; u < 4; ++u) { b[u].x += v[u].x; b[u].y += v[u].y; b[u].z += v[u].z; b[u].w += v[u].w; }
    }
    for (; p < S.P; p += 16) {
      const float4 v = *reinterpret_cast<const float4*>(S.part + (size_t)p * k + c0);
      b[0].x += v.x; b[0].y += v.y; b[0].z += v.z; b[0].w += v.w;
    }
    a.x = (b[0].x + b[1].x) + (b[2].x + b[3].x);
    a.y = (b[0].y + b[1].y) + (b[2].y + b[3].y);
    a.z = (b[0].z + b[1].z) + (b[2].z + b[3].z);
    a.w = (b[0].w + b[1].w) + (b[2].w + b[3].w);
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
      if (S.accumulate) t += bf2f(S.out[c]);
      S.out[c] = f2bf(t);
    }
  }
}

}  // namespace

#ifndef DLTB_COLPART_RPP
#define DLTB_COLPART_RPP 16     // rows per partial (per workgroup)
#endif
#ifndef DLTB_COLPART_PMAX
#define DLTB_COLPART_PMAX 128   // partial rows at most
#endif
int dltb_colpart_partials(int N) {
  int P = N / DLTB_COLPART_RPP;
  if (P < 1) P = 1;
  if (P > DLTB_COLPART_PMAX) P = DLTB_COLPART_PMAX;
  return P;
}

void dltb_colpart(const DltbColPartSeg* segs, int nseg, int P, uint32_t thr16, float drop_scale,
                  const int64_t* seed, hipStream_t st) {
  ColPartArgs A{};
  int maxk = 0;
  for (int i = 0; i < nseg; ++i) {
    A.seg[i] = segs[i];
    maxk = segs[i].k > maxk ? segs[i].k : maxk;
  }
  A.P = P;
  A.thr16 = thr16;
  A.drop_scale = drop_scale;
  A.seed_ptr = seed;
  hipLaunchKernelGGL(colpart_kernel, dim3(cdiv(maxk, 512), P, nseg), dim3(256), 0, st, A);
}

void dltb_colreduce_multi(const DltbColRedSeg* segs, int nseg, hipStream_t st) {
  ColRedArgs A{};
  int maxk = 0;
  for (int i = 0; i < nseg; ++i) {
    A.seg[i] = segs[i];
    maxk = segs[i].k > maxk ? segs[i].k : maxk;
  }
  hipLaunchKernelGGL(colreduce_multi_kernel, dim3(cdiv(maxk, 64), nseg), dim3(256), 0, st, A);
}
