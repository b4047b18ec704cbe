// Fused softmax cross-entropy forward + backward for gfx950 (F.cross_entropy with
// ignore_index, train_harness.py:99-103).
//
// One 512-thread workgroup per row; the whole bf16 row (V = 32000 -> 8 x 16-byte vectors per
// thread) stays in registers, so logits are read from HBM exactly once:
//     loss[r]      = logsumexp(z_r) - z_r[t_r]              (0 for ignored rows)
//     z_r (in place) <- softmax(z_r) - onehot(t_r)           (unscaled dlogits; 0 for ignored)
// The 1/count mean-reduction and the incoming grad_output are applied by the caller as a device
// scalar folded into the head GEMMs, so no host sync is needed anywhere.
#include "common.h"

namespace {

template <int VPT>
__global__ __launch_bounds__(512) void xent_kernel(bf16_t* __restrict__ logits,
                                                  const int64_t* __restrict__ targets,
                                                  float* __restrict__ loss, int V,
                                                  int64_t ignore_index) {
  __shared__ float red[8], red2[8];
  __shared__ float s_tlogit;
  const int row = blockIdx.x;
  bf16_t* z = logits + (long)row * V;
  const int64_t t = targets[row];
  const bool valid = (t != ignore_index) && t >= 0 && t < V;
  if (threadIdx.x == 0) s_tlogit = valid ? bf2f(z[t]) : 0.f;
  const int nvec = V >> 3;
  // one pass over the row: per-thread max m_t and e = exp(z - m_t) kept in registers, then ONE
  // block reduction of (m_t, sum e) pairs (online-softmax merge); the output rescales e by
  // exp(m_t - m) / sum instead of recomputing the exponentials
  float e[VPT][8];
  float mt = -INFINITY;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int i = j * 512 + threadIdx.x;
    if (i < nvec) {
      unpack8(ld16<uint4>(z + i * 8), e[j]);
#pragma unroll
      for (int k = 0; k < 8; ++k) mt = fmaxf(mt, e[j][k]);
    }
  }
  float st = 0.f;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int i = j * 512 + threadIdx.x;
    if (i < nvec) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        e[j][k] = __expf(e[j][k] - mt);
        st += e[j][k];
      }
    }
  }
  // (m, s) pairs: wave butterfly, then the 8 waves through LDS (fixed order)
  float m = mt, sm = st;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const float mo = __shfl_xor(m, off);
    const float so = __shfl_xor(sm, off);
    const float mn = fmaxf(m, mo);
    sm = (m == -INFINITY ? 0.f : sm * __expf(m - mn)) + (mo == -INFINITY ? 0.f : so * __expf(mo - mn));
    m = mn;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    red[wid] = m;
    red2[wid] = sm;
  }
  __syncthreads();
  float M = -INFINITY;
#pragma unroll
  for (int w = 0; w < 8; ++w) M = fmaxf(M, red[w]);
  float S = 0.f;
#pragma unroll
  for (int w = 0; w < 8; ++w) S += red[w] == -INFINITY ? 0.f : red2[w] * __expf(red[w] - M);
  if (threadIdx.x == 0) loss[row] = valid ? (M + __logf(S) - s_tlogit) : 0.f;
  const float scale = mt == -INFINITY ? 0.f : __expf(mt - M) / S;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int i = j * 512 + threadIdx.x;
    if (i < nvec) {
      float f[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float p = valid ? e[j][k] * scale : 0.f;
        if (valid && i * 8 + k == t) p -= 1.f;
        f[k] = p;
      }
      *reinterpret_cast<uint4*>(z + i * 8) = pack8(f);
    }
  }
}

// mean over non-ignored rows in one 1024-thread workgroup (fixed summation order):
//   out[0] = sum(loss) / max(count, 1),  out[1] = max(count, 1)
__global__ __launch_bounds__(1024) void xent_mean_kernel(const float* __restrict__ loss,
                                                        const int64_t* __restrict__ targets, int N,
                                                        int64_t ignore_index, float* __restrict__ out) {
  __shared__ float red[16];
  float s = 0.f, c = 0.f;
  for (int i = threadIdx.x; i < N; i += 1024) {
    s += loss[i];
    c += targets[i] != ignore_index ? 1.f : 0.f;
  }
  s = block_sum(s, red);
  c = block_sum(c, red);
  if (threadIdx.x == 0) {
    c = fmaxf(c, 1.f);
    out[0] = s / c;
    out[1] = c;
  }
}

}  // namespace

void dltb_xent_mean(const float* loss, const int64_t* targets, int N, int64_t ignore_index, float* out,
                    hipStream_t st) {
  hipLaunchKernelGGL(xent_mean_kernel, dim3(1), dim3(1024), 0, st, loss, targets, N, ignore_index, out);
}

void dltb_xent_fwd_bwd(void* logits, const int64_t* targets, float* loss, int N, int V,
                       int64_t ignore_index, hipStream_t st) {
  const int vpt = cdiv(V / 8, 512);
#define DLTB_XE(K)                                                                              \
  hipLaunchKernelGGL(xent_kernel<K>, dim3(N), dim3(512), 0, st, (bf16_t*)logits, targets, loss, \
                     V, ignore_index)
  if (vpt <= 1) DLTB_XE(1);
  else if (vpt <= 2) DLTB_XE(2);
  else if (vpt <= 4) DLTB_XE(4);
  else if (vpt <= 8) DLTB_XE(8);
  else if (vpt <= 16) DLTB_XE(16);
  else DLTB_XE(32);
#undef DLTB_XE
}
