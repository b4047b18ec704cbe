// Packed attention-dropout keep bits: the device body shared by attention.hip's attn_mask_kernel
// and norm.hip's norm_fwd_mask_kernel (the mask of a block generated in the same launch as its
// first LayerNorm: the VALU-bound hash and the latency-bound row norm fill each other's idle
// issue slots).
//
// word (bh, t, h, q) at ((bh*nT + t)*2 + h)*T + q; bit mask_bit(n, i) <-> key 64t + 32n + (i&3) + 8(i>>2) + 4h
// (the lane layout of the attention kernels' S tiles; see attention.hip).  Score pair j = 8n + (i>>1)
// (the two probabilities one v_cvt_pk_bf16_f32 packs) sits at bits 15 - j (even i) and 31 - j (odd i):
// after a left shift by j both are sign bits of their 16-bit halves, so one v_perm_b32 turns them
// into the pair's 0x0000/0xFFFF keep masks and the forward drops probabilities on the packed bf16
// P operand (shift + perm + and per PAIR instead of bfe + and per score).
#pragma once
#include "common.h"

constexpr int kMaskKeyTile = 64;   // keys per packed tile (attention.hip kTile)

// bit of score register i (0..15) of key sub-tile n (0, 1) in a packed keep word
constexpr uint32_t mask_bit(int n, int i) {
  return (uint32_t)((i & 1) ? 31 - (8 * n + (i >> 1)) : 15 - (8 * n + (i >> 1)));
}

// one thread = one query row q of tile group g = (bh * nT + t) * 2 + h; 32 keep decisions.  g is
// uniform over the calling block (both callers), and every thread of the block must call: the 16
// column-pair keys of the tile are mixed once per block (16 lanes, one VALU pass) and read from LDS.
DLTB_DEV void attn_mask_word(uint32_t* __restrict__ mask, int T, uint32_t thr16, const int64_t* __restrict__ seed_ptr,
                             int64_t site, int q, uint32_t g) {
  __shared__ __attribute__((aligned(16))) uint32_t ckey[16];
  const int nT = T / kMaskKeyTile;
  const int h = g & 1;
  const int t = (g >> 1) % nT;
  const uint32_t bh = (g >> 1) / nT;
  const uint64_t seed = site_seed(seed_ptr, site);
  if (threadIdx.x < 16) {                  // pair k: register pair j = k of key sub-tile n = k / 8
    const int k = threadIdx.x, n = k >> 3, i = 2 * (k & 7);
    ckey[k] = rng_attn_col_key(seed, (uint32_t)(t * kMaskKeyTile + 32 * n + (i & 3) + 8 * (i >> 2) + 4 * h));
  }
  __syncthreads();
  if (q >= T) return;
  uint32_t rk = rng_row_key(seed, bh * (uint32_t)T + q);
  asm("" : "+v"(rk));     // materialised once (else its last xor-shift is re-done per pair)
  uint32_t bits = 0xFFFFFFFFu;                               // thr16 == 0: keep everything
  if (thr16 != 0) {
    // one hash covers a key pair (i, i+1) of register pair j = 8n + i/2, whose keep bits live at
    // 15 - j and 31 - j: both 16-bit halves compared at once, (h - (thr - 1)) saturated then
    // min'ed with 1 gives 0 / 1 per half, shifted into place by one v_lshl_or_b32
    const uint32_t tm2 = (thr16 - 1u) * 0x10001u, one2 = 0x10001u;
    bits = 0;
    const uint4* ck4 = reinterpret_cast<const uint4*>(ckey);
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const uint4 ck = ck4[2 * n + c];                       // keys of pairs 8n + 4c .. + 3
        const uint32_t cks[4] = {ck.x, ck.y, ck.z, ck.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 2 * (4 * c + e);
          const uint32_t hsh = rng_attn_pair(rk, cks[e]);
          uint32_t kk;
          asm("v_pk_sub_u16 %0, %1, %2 clamp\n\tv_pk_min_u16 %0, %0, %3"
              : "=&v"(kk) : "v"(hsh), "v"(tm2), "v"(one2));
          static_assert(mask_bit(0, 1) == mask_bit(0, 0) + 16, "pair bits 16 apart");
          bits |= kk << mask_bit(n, i);
        }
      }
  }
  mask[(size_t)g * T + q] = bits;
}
