// Token + learned-position embedding with fused dropout (train_harness.py:85-89) and its
// backward for gfx950.
//
// forward : x[r, :] = dropout(wte[idx[r]] + wpe[r % T])       one wave per token row
// backward: g = dropout_mask(dx) * 1/(1-p)
//           dwpe[t]   (+)= sum_b g[b*T + t]                      one wave per position
//           dwte[v]   +=  sum_{r : idx[r] = v} g[r]              deterministic segmented sum over
//                                                               the sorted token ids (no atomics)
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void embed_fwd_kernel(
    const int64_t* __restrict__ idx, const bf16_t* __restrict__ wte, const bf16_t* __restrict__ wpe,
    bf16_t* __restrict__ x, int N, int T, int d, uint32_t thr16, float scale,
    const int64_t* __restrict__ seed_ptr, int64_t site) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  const long tok = idx[row];
  const int t = row % T;
  uint64_t seed = 0;
  uint32_t rk = 0;
  if (thr16) {
    seed = site_seed(seed_ptr, site);
    rk = rng_row_key(seed, (uint32_t)row);
  }
  const bf16_t* a = wte + tok * d;
  const bf16_t* b = wpe + (long)t * d;
  bf16_t* o = x + (long)row * d;
  for (int c = lane * 8; c < d; c += 512) {
    float va[8], vb[8];
    unpack8(ld16<uint4>(a + c), va);
    unpack8(ld16<uint4>(b + c), vb);
#pragma unroll
    for (int e = 0; e < 8; ++e) va[e] += vb[e];
    if (thr16) {
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        const uint32_t h = rng_pair(rk, rng_col_key(seed, (uint32_t)(c + e)));
        va[e] = keep_lo(h, thr16) ? va[e] * scale : 0.f;
        va[e + 1] = keep_hi(h, thr16) ? va[e + 1] * scale : 0.f;
      }
    }
    *reinterpret_cast<uint4*>(o + c) = pack8(va);
  }
}

DLTB_DEV void load_masked(const bf16_t* __restrict__ dx, int row, int c, int d, uint32_t thr16,
                          float scale, uint64_t seed, float* v) {
  unpack8(ld16<uint4>(dx + (long)row * d + c), v);
  if (thr16) {
    const uint32_t rk = rng_row_key(seed, (uint32_t)row);
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      const uint32_t h = rng_pair(rk, rng_col_key(seed, (uint32_t)(c + e)));
      v[e] = keep_lo(h, thr16) ? v[e] * scale : 0.f;
      v[e + 1] = keep_hi(h, thr16) ? v[e + 1] * scale : 0.f;
    }
  }
}

// one wave per position t in [0, P) (P = wpe rows); rows >= T get zeros unless accumulating
__global__ __launch_bounds__(256) void embed_bwd_pos_kernel(
    const bf16_t* __restrict__ dx, bf16_t* __restrict__ dwpe, int B, int T, int P, int d,
    int accumulate, uint32_t thr16, float scale, const int64_t* __restrict__ seed_ptr,
    int64_t site) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= P) return;
  const uint64_t seed = thr16 ? site_seed(seed_ptr, site) : 0ull;
  for (int c = lane * 8; c < d; c += 512) {
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    if (t < T) {
      for (int b = 0; b < B; ++b) {
        float v[8];
        load_masked(dx, b * T + t, c, d, thr16, scale, seed, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += v[e];
      }
    }
    bf16_t* o = dwpe + (long)t * d + c;
    if (accumulate) {
      float old[8];
      unpack8(ld16<uint4>(o), old);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += old[e];
    }
    *reinterpret_cast<uint4*>(o) = pack8(acc);
  }
}

// sorted_ids[i] (ascending), perm[i] = original row.  One wave per sorted position; the first
// position of each run of equal ids sums the run and adds it to dwte[id].
__global__ __launch_bounds__(256) void embed_bwd_tok_kernel(
    const bf16_t* __restrict__ dx, const int64_t* __restrict__ sorted_ids,
    const int64_t* __restrict__ perm, bf16_t* __restrict__ dwte, int N, int d, long V, uint32_t thr16,
    float scale, const int64_t* __restrict__ seed_ptr, int64_t site) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= N) return;
  const long id = sorted_ids[i];
  if (i > 0 && sorted_ids[i - 1] == id) return;
  if (id < 0 || id >= V) return;   // ignore_index style padding ids; never a row outside the table
  int j_end = i + 1;
  while (j_end < N && sorted_ids[j_end] == id) ++j_end;
  const uint64_t seed = thr16 ? site_seed(seed_ptr, site) : 0ull;
  for (int c = lane * 8; c < d; c += 512) {
    float acc[8];
    unpack8(ld16<uint4>(dwte + id * d + c), acc);
    for (int j = i; j < j_end; ++j) {
      float v[8];
      load_masked(dx, (int)perm[j], c, d, thr16, scale, seed, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
    *reinterpret_cast<uint4*>(dwte + id * d + c) = pack8(acc);
  }
}

// Sort-free variant for N <= kScanMaxRows (one micro-batch): one wave per position i.  The wave
// first checks (64 ids per step, ballot) whether an earlier position holds the same id - if so it
// exits - so exactly one wave per distinct id survives; it then sums the rows of every later
// position with that id in ascending order (deterministic) and adds the sum to dwte[id].  The id
// scans read 8 * N bytes per wave from L1/L2; at N = 2048 that replaces a torch radix sort plus its
// index bookkeeping (~35 us) by nothing.
constexpr int kScanMaxRows = 4096;     // beyond: the sort path (the duplicate scan is O(N^2 / 64))
constexpr int kScanMaxChunks = 8;     // d <= 8 x 512 = 4096

__global__ __launch_bounds__(256) void embed_bwd_tok_scan_kernel(
    const bf16_t* __restrict__ dx, const int64_t* __restrict__ ids, bf16_t* __restrict__ dwte, int N,
    int d, long V, uint32_t thr16, float scale, const int64_t* __restrict__ seed_ptr, int64_t site) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= N) return;
  const long id = ids[i];
  if (id < 0 || id >= V) return;
  DLTB_DCHECK(d % 8 == 0 && d <= kScanMaxChunks * 512);
  for (int base = 0; base < i; base += 64) {            // an earlier duplicate owns this id
    const int j = base + lane;
    if (__ballot(j < i && ids[j] == id)) return;
  }
  const uint64_t seed = thr16 ? site_seed(seed_ptr, site) : 0ull;
  // the id scan runs with all 64 lanes active (ballot), the row chunks per lane below it
  float acc[kScanMaxChunks][8];
#pragma unroll
  for (int cc = 0; cc < kScanMaxChunks; ++cc) {
    const int c = cc * 512 + lane * 8;
    if (c < d) unpack8(ld16<uint4>(dwte + id * d + c), acc[cc]);
  }
  for (int base = i; base < N; base += 64) {
    const int j = base + lane;
    uint64_t m = __ballot(j < N && ids[j] == id);
    while (m) {
      const int jj = base + __builtin_ctzll(m);
      m &= m - 1;
#pragma unroll
      for (int cc = 0; cc < kScanMaxChunks; ++cc) {
        const int c = cc * 512 + lane * 8;
        if (c < d) {
          float v[8];
          load_masked(dx, jj, c, d, thr16, scale, seed, v);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[cc][e] += v[e];
        }
      }
    }
  }
#pragma unroll
  for (int cc = 0; cc < kScanMaxChunks; ++cc) {
    const int c = cc * 512 + lane * 8;
    if (c < d) *reinterpret_cast<uint4*>(dwte + id * d + c) = pack8(acc[cc]);
  }
}

}  // namespace

bool dltb_embed_bwd_tok_scan(const void* dx, const int64_t* ids, void* dwte, int N, int d, long V,
                             uint32_t thr16, float scale, const int64_t* seed, int64_t site,
                             hipStream_t st) {
  if (N > kScanMaxRows || d > kScanMaxChunks * 512 || d % 8) return false;
  hipLaunchKernelGGL(embed_bwd_tok_scan_kernel, dim3(cdiv(N, 4)), dim3(256), 0, st,
                     (const bf16_t*)dx, ids, (bf16_t*)dwte, N, d, V, thr16, scale, seed, site);
  return true;
}

void dltb_embed_fwd(const int64_t* idx, const void* wte, const void* wpe, void* x, int N, int T,
                    int d, uint32_t thr16, float scale, const int64_t* seed, int64_t site,
                    hipStream_t st) {
  hipLaunchKernelGGL(embed_fwd_kernel, dim3(cdiv(N, 4)), dim3(256), 0, st, idx,
                     (const bf16_t*)wte, (const bf16_t*)wpe, (bf16_t*)x, N, T, d, thr16, scale,
                     seed, site);
}

void dltb_embed_bwd_pos(const void* dx, void* dwpe, int B, int T, int P, int d, int accumulate,
                        uint32_t thr16, float scale, const int64_t* seed, int64_t site,
                        hipStream_t st) {
  hipLaunchKernelGGL(embed_bwd_pos_kernel, dim3(cdiv(P, 4)), dim3(256), 0, st,
                     (const bf16_t*)dx, (bf16_t*)dwpe, B, T, P, d, accumulate, thr16, scale, seed,
                     site);
}

void dltb_embed_bwd_tok(const void* dx, const int64_t* sorted_ids, const int64_t* perm,
                        void* dwte, int N, int d, long V, uint32_t thr16, float scale,
                        const int64_t* seed, int64_t site, hipStream_t st) {
  hipLaunchKernelGGL(embed_bwd_tok_kernel, dim3(cdiv(N, 4)), dim3(256), 0, st,
                     (const bf16_t*)dx, sorted_ids, perm, (bf16_t*)dwte, N, d, V, thr16, scale, seed,
                     site);
}
