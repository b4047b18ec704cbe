// Shared device helpers for the dltb CDNA4 (gfx950) kernels.
//
// * bf16 <-> f32 conversion (hardware v_cvt_pk_bf16_f32 via the __bf16 type)
// * 16-byte vector load/store helpers (Guideline 13: never scalar bf16 loads)
// * 64-lane wave reductions (CDNA wave = 64 lanes)
// * the counter-hash dropout RNG, bit-identical to dltb/ops/rng.py
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DLTB_DEV __device__ __forceinline__

// Device-side bound checks of the checked build (csrc/build.py --debug => DLTB_DEBUG=1): print the
// failing condition with the kernel and block, then trap.  Compiled out of release builds.
#if defined(DLTB_DEBUG) && DLTB_DEBUG
#define DLTB_DCHECK(cond)                                                                        \
  do {                                                                                           \
    if (!(cond)) {                                                                               \
      printf("[dltb DCHECK] %s failed in %s (block %d,%d thread %d)\n", #cond, __func__,         \
             (int)blockIdx.x, (int)blockIdx.y, (int)threadIdx.x);                                \
      __builtin_trap();                                                                          \
    }                                                                                            \
  } while (0)
#else
#define DLTB_DCHECK(cond) \
  do {                    \
  } while (0)
#endif

// 16-bit storage format of this translation unit.  Every kernel file is compiled twice
// (csrc/build.py): DLTB_F16=0 -> bf16 (the default compute dtype), DLTB_F16=1 -> IEEE fp16 (the
// reference's DDP/FSDP autocast precision; host entry points renamed dltb_*_f16).  Tensors are
// moved as raw 16-bit words (bf16_t) and converted to fp32 at the arithmetic by the helpers below,
// so the kernel bodies are format-independent; the MFMA operand type follows h16_t.
#ifndef DLTB_F16
#define DLTB_F16 0
#endif
typedef uint16_t bf16_t;                                     // raw 16-bit float bits (bf16 or fp16)
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));    // MFMA A/B fragment (4 VGPRs)
typedef short bf16x4 __attribute__((ext_vector_type(4)));

#if DLTB_F16
typedef _Float16 h16_t;
DLTB_DEV float bf2f(bf16_t u) { return (float)__builtin_bit_cast(_Float16, u); }
DLTB_DEV bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (_Float16)f); }
DLTB_DEV float lo_bf(uint32_t w) { return bf2f((bf16_t)(w & 0xFFFFu)); }
DLTB_DEV float hi_bf(uint32_t w) { return bf2f((bf16_t)(w >> 16)); }
#else
typedef __bf16 h16_t;
DLTB_DEV float bf2f(bf16_t u) { return __uint_as_float(((uint32_t)u) << 16); }
DLTB_DEV bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}
DLTB_DEV float lo_bf(uint32_t w) { return __uint_as_float(w << 16); }
DLTB_DEV float hi_bf(uint32_t w) { return __uint_as_float(w & 0xFFFF0000u); }
#endif
// two floats -> packed 16-bit x2 in one dword (low = a)
DLTB_DEV uint32_t pack_bf2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

// unpack 8 bf16 held in a uint4 into floats
DLTB_DEV void unpack8(const uint4& v, float* f) {
  f[0] = lo_bf(v.x); f[1] = hi_bf(v.x);
  f[2] = lo_bf(v.y); f[3] = hi_bf(v.y);
  f[4] = lo_bf(v.z); f[5] = hi_bf(v.z);
  f[6] = lo_bf(v.w); f[7] = hi_bf(v.w);
}
DLTB_DEV uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack_bf2(f[0], f[1]);
  v.y = pack_bf2(f[2], f[3]);
  v.z = pack_bf2(f[4], f[5]);
  v.w = pack_bf2(f[6], f[7]);
  return v;
}

template <typename T>
DLTB_DEV T ld16(const void* p) { return *reinterpret_cast<const T*>(p); }

// ---------------------------------------------------------------- wave / block reductions
DLTB_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
DLTB_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// block-wide sum; `red` must hold >= (blockDim.x / 64) floats of LDS
DLTB_DEV float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}
DLTB_DEV float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = -INFINITY;
  for (int i = 0; i < nw; ++i) t = fmaxf(t, red[i]);
  return t;
}

// ---------------------------------------------------------------- GELU (erf form, nn.GELU default)
// erf via Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far below bf16 resolution): one v_rcp,
// one v_exp and 6 FMAs instead of the libm erff polynomial chain -- the GELU kernels become
// HBM-bound.  The derivative pdf term reuses the same exp(-x^2/2).
DLTB_DEV float erf_fast(float x, float* e_out = nullptr) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.f));
  const float e = __expf(-ax * ax);
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float y = 1.f - p * t * e;
  if (e_out) *e_out = e;
  return copysignf(y, x);
}
DLTB_DEV float gelu_fwd_f(float x) { return 0.5f * x * (1.f + erf_fast(x * 0.70710678118654752f)); }
DLTB_DEV float gelu_grad_f(float x) {
  float e;                                                  // e = exp(-x^2 / 2)
  const float cdf = 0.5f * (1.f + erf_fast(x * 0.70710678118654752f, &e));
  return cdf + x * 0.39894228040143268f * e;
}

// ---------------------------------------------------------------- dropout RNG (see ops/rng.py)
#define DLTB_C_ROW 0x9E3779B1u
#define DLTB_C_COL 0x85EBCA77u
#define DLTB_GOLDEN64 0x9E3779B97F4A7C15ull

DLTB_DEV uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
DLTB_DEV uint64_t splitmix64(uint64_t x) {
  x += DLTB_GOLDEN64;
  uint64_t z = x;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// seed of one dropout site: splitmix64(step_seed + site * golden)
DLTB_DEV uint64_t site_seed(const int64_t* seed_ptr, int64_t site) {
  return splitmix64((uint64_t)(*seed_ptr) + (uint64_t)site * DLTB_GOLDEN64);
}
DLTB_DEV uint32_t rng_row_key(uint64_t seed, uint32_t row) {
  return fmix32(row * DLTB_C_ROW + (uint32_t)(seed >> 32));
}
DLTB_DEV uint32_t rng_col_key(uint64_t seed, uint32_t col) {
  return (col >> 1) * DLTB_C_COL + (uint32_t)seed;
}
// hash covering the column pair (col & ~1, col | 1)
DLTB_DEV uint32_t rng_pair(uint32_t row_key, uint32_t col_key) { return fmix32(row_key ^ col_key); }
// Attention-probability dropout (the packed mask of attn_mask.h, 2/3 of all dropout decisions of a TinyGPT
// step): the column key is mixed by its own fmix32 -- wave-uniform in the mask generators, so scalar ALU work --
// and each (row, column pair) needs ONE multiply-xorshift round on the two independent 32-bit hashes: 3 VALU
// per pair instead of fmix32's 6 (ops/rng.py attn_keep_mask; the statistical checks are in tests/test_ref_ops.py)
DLTB_DEV uint32_t rng_attn_col_key(uint64_t seed, uint32_t col) { return fmix32(rng_col_key(seed, col)); }
DLTB_DEV uint32_t rng_attn_pair(uint32_t row_key, uint32_t col_mixed) {
  const uint32_t h = (row_key ^ col_mixed) * 0x85EBCA6Bu;
  return h ^ (h >> 16);
}
DLTB_DEV bool rng_keep(uint32_t x, uint32_t col, uint32_t thr16) {
  uint32_t r = (col & 1u) ? (x >> 16) : (x & 0xFFFFu);
  return r >= thr16;
}
DLTB_DEV bool keep_lo(uint32_t x, uint32_t thr16) { return (x & 0xFFFFu) >= thr16; }
DLTB_DEV bool keep_hi(uint32_t x, uint32_t thr16) { return (x >> 16) >= thr16; }

static inline uint32_t host_drop_threshold(float p) {
  double t = (double)p * 65536.0 + 0.5;
  uint32_t v = (uint32_t)t;
  return v > 65536u ? 65536u : v;
}

// XCD-grouped tile index of workgroup L in a grid of `tiles`: the dispatcher deals consecutive workgroups to
// the 8 XCDs round robin, so XCD x = L & 7 gets the contiguous index range
// [x (tiles / 8) + min(x, tiles % 8), ... + tiles / 8 + (x < tiles % 8)) -- neighbouring tiles (which share
// operand slabs) meet in one XCD's L2.  A bijection on [0, tiles) for any tile count (performance only).
DLTB_DEV int xcd_grouped(int L, int tiles) {
  const int x = L & 7, q = tiles >> 3, r = tiles & 7;
  return x * q + (x < r ? x : r) + (L >> 3);
}

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }
