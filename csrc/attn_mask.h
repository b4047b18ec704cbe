// Packed attention-dropout keep bits: the device body shared by attention.hip's attn_mask_kernel
// and norm.hip's norm_fwd_mask_kernel (the mask of a block generated in the same launch as its
// first LayerNorm: the VALU-bound hash and the latency-bound row norm fill each other's idle
// issue slots).
//
// word (bh, t, h, q) at ((bh*nT + t)*2 + h)*T + q; bit 16n + i <-> key 64t + 32n + (i&3) + 8(i>>2) + 4h
// (the lane layout of the attention kernels' S tiles; see attention.hip).
#pragma once
#include "common.h"

constexpr int kMaskKeyTile = 64;   // keys per packed tile (attention.hip kTile)

// one thread = one query row q of tile group g = (bh * nT + t) * 2 + h; 32 keep decisions
DLTB_DEV void attn_mask_word(uint32_t* __restrict__ mask, int T, uint32_t thr16, const int64_t* __restrict__ seed_ptr,
                             int64_t site, int q, uint32_t g) {
  if (q >= T) return;
  const int nT = T / kMaskKeyTile;
  const int h = g & 1;
  const int t = (g >> 1) % nT;
  const uint32_t bh = (g >> 1) / nT;
  const uint64_t seed = site_seed(seed_ptr, site);
  const uint32_t rk = rng_row_key(seed, bh * (uint32_t)T + q);
  uint32_t bits = 0;
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
      const uint32_t key = (uint32_t)(t * kMaskKeyTile + 32 * n + (i & 3) + 8 * (i >> 2) + 4 * h);
      const uint32_t hsh = rng_pair(rk, rng_col_key(seed, key));
      bits |= (keep_lo(hsh, thr16) ? 1u : 0u) << (16 * n + i);
      bits |= (keep_hi(hsh, thr16) ? 1u : 0u) << (16 * n + i + 1);
    }
  mask[(size_t)g * T + q] = bits;
}
