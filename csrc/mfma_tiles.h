// MFMA / LDS tile helpers shared by the attention and GEMM kernels (gfx950, CDNA4).
//
// * v_mfma_f32_32x32x16_bf16 wrapper: C[i][j] += sum_k A[i][k] B[k][j]; operand fragments are 8 bf16
//   (lane l: row/col l & 31, k-half l >> 5), the accumulator holds column j = l & 31 and rows
//   (r & 3) + 8 (r >> 2) + 4 (l >> 5) of register r.
// * LDS tile images with rows of D bf16 (D = 64: 128-byte rows, D = 128: 256-byte rows) and a
//   16-byte-chunk XOR swizzle that makes both read patterns bank-conflict free:
//     row_frag - ds_read_b128 of 8 consecutive elements of one row   (K-contiguous operands)
//     tr_frag  - 2 x ds_read_b64_tr_b16: 8 elements of one column     (K-strided operands; the k
//                order is permuted as (j & 3) + 8 (j >> 2) + 4 h, identical for both operands)
// * GldsTile: LDS-DMA (global_load_lds_dwordx4) fill of such an image with the swizzle applied to
//   the SOURCE address (the LDS side of an LDS-DMA is lane-linear, 1 KiB per wave-instruction).
#pragma once
#include "common.h"

namespace {

typedef h16_t bfx8 __attribute__((ext_vector_type(8)));      // 8 x (bf16 | fp16): one A/B fragment
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

DLTB_DEV f32x16 mfma32(bfx8 a, bfx8 b, f32x16 c) {
#if DLTB_F16
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
#else
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
#endif
}

template <int D>
DLTB_DEV int swz(int row) {
  if constexpr (D == 32) return (row >> 2) & 3;   // 64-byte rows: 4 rows per 256-byte bank row
  if constexpr (D == 64) return (((row >> 1) & 1) << 2) | ((row >> 2) & 3);
  else return ((row & 3) << 2) | ((row >> 2) & 3);
}
template <int D>
DLTB_DEV int toff(int row, int ch) {   // byte offset of 16-byte chunk `ch` of tile row `row`
  return row * (D * 2) + ((ch ^ swz<D>(row)) << 4);
}

// A-operand row fragment: lane (r, h) <- tile[row][16s + 8h .. +7] (chunk 2s + h)
template <int D>
DLTB_DEV bfx8 row_frag(const char* tile, int row, int ch) {
  uint4 v = *reinterpret_cast<const uint4*>(tile + toff<D>(row, ch));
  return __builtin_bit_cast(bfx8, v);
}

// A-operand transposed fragment for  Y = A * X  where X is a 32x32 accumulator whose rows are
// tile rows [row_base, row_base + 16) of k-step s.  Lane (r = lane & 31, h = lane >> 5) gets
// element j = tile[row_base + 8(j>>2) + 4h + (j&3)][col_base + r], matching the permuted k order
// of an accumulator used as the B operand.
template <int D>
DLTB_DEV bfx8 tr_frag(const char* tile, int row_base, int col_base, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int row = row_base + 4 * (g >> 1) + (i >> 2);
  const int col = col_base + 16 * (g & 1) + 4 * (i & 3);
  const char* p0 = tile + toff<D>(row, col >> 3) + (col & 7) * 2;
  const char* p1 = tile + toff<D>(row + 8, col >> 3) + (col & 7) * 2;
  s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p0);
  s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p1);
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 c = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bfx8, c);
}

// Hoisted addressing.  The swizzle only reads row bits 0..3, so a fragment whose tile row is
// (multiple of 16) + (lane part) has the byte offset  16-row-aligned base * (2 D) + lane offset:
// the lane offset is loop-invariant (a VGPR computed once), the row base a compile-time constant
// the compiler folds into the ds_read's immediate offset field.  Per tile that leaves one VALU add
// per distinct lane offset (stage base + offset) instead of address arithmetic per LDS read.
template <int D>
DLTB_DEV uint32_t row_lane_off(int lane_row, int ch) { return (uint32_t)toff<D>(lane_row, ch); }
template <int D>
DLTB_DEV uint32_t tr_lane_off(int col_base, int half, int lane) {   // tr_frag's p0 (half 0) / p1 (half 1)
  const int g = lane >> 4, i = lane & 15;
  const int row = 4 * (g >> 1) + (i >> 2) + 8 * half;
  const int col = col_base + 16 * (g & 1) + 4 * (i & 3);
  return (uint32_t)(toff<D>(row, col >> 3) + (col & 7) * 2);
}
typedef __attribute__((address_space(3))) const char lds_cchar;
typedef __attribute__((address_space(3))) const uint4 lds_u4;
// 32-bit LDS address of a pointer into dynamic shared memory
DLTB_DEV uint32_t lds_addr(const void* p) { return (uint32_t)(size_t)(lds_cchar*)p; }
// stage base (wave-uniform, SGPR) + lane offset in one v_add the compiler cannot re-associate: the
// fragment reads below then carry their row constants in the ds_read immediate offset instead of a
// per-read subtract + add chain (LSR re-derives one address per read otherwise)
DLTB_DEV uint32_t lane_addr(uint32_t sbase, uint32_t off) {
  uint32_t a;
  asm("v_add_u32 %0, %1, %2" : "=v"(a) : "s"(sbase), "v"(off));
  return a;
}
template <int OFF>
DLTB_DEV bfx8 row_frag_at(uint32_t a) { return __builtin_bit_cast(bfx8, *(lds_u4*)(size_t)(a + OFF)); }
// tr_frag(tile, row_base, col_base, lane) == tr_frag_at<row_base * 2 D>(base + tr_lane_off(col_base, 0),
// base + tr_lane_off(col_base, 1)) for row_base % 16 == 0
template <int OFF>
DLTB_DEV bfx8 tr_frag_at(uint32_t a0, uint32_t a1) {
  s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(size_t)(a0 + OFF));
  s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(size_t)(a1 + OFF));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 c = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bfx8, c);
}

// ROWS-row tile of D-element rows filled by LDS-DMA from a row-major global matrix (rows
// row0 .. row0 + ROWS - 1, columns col0 .. col0 + D - 1 of `base`, row stride `stride`) by 4 waves.
// Completion: a __syncthreads() (which waits vmcnt(0)) before anyone reads the tile.
// One LDS-DMA instruction issued from inline asm: invisible to hipcc's waitcnt bookkeeping, so the
// compiler does NOT insert a vmcnt(0) before the next LDS read (it would drain a multi-stage ring).
// The caller retires it with a counted s_waitcnt vmcnt (gemm.hip wait_vm) + s_barrier.
DLTB_DEV void glds16_asm(const void* gsrc, const void* lds_dst) {
  const uint32_t lds = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)lds_dst);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds)
               : "memory");
}

// 4-byte LDS-DMA from inline asm (one dword per lane -> 256 contiguous LDS bytes per wave).
DLTB_DEV void glds4_asm(const void* gsrc, const void* lds_dst) {
  const uint32_t lds = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)lds_dst);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds)
               : "memory");
}

// Scalar-base forms: address = wave-uniform 64-bit base (SGPR pair, advanced per tile by SALU) +
// a loop-invariant per-lane 32-bit byte offset (VGPR) -- no per-tile VALU address arithmetic.
DLTB_DEV uint64_t uniform_ptr(const void* p) {
  const uint64_t b = (uint64_t)(uintptr_t)p;
  // (readfirstlane returns int: widen through uint32_t, never sign-extend the low half)
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
  return ((uint64_t)hi << 32) | (uint64_t)lo;
}
DLTB_DEV void glds16_sv(const void* sbase, uint32_t voff, const void* lds_dst) {
  const uint32_t lds = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)lds_dst);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(uniform_ptr(sbase)), "s"(lds)
               : "memory");
}
DLTB_DEV void glds4_sv(const void* sbase, uint32_t voff, const void* lds_dst) {
  const uint32_t lds = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)lds_dst);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dword %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(uniform_ptr(sbase)), "s"(lds)
               : "memory");
}

// s_waitcnt vmcnt(N) only (gfx9 encoding: vmcnt[3:0] | vmcnt[5:4] << 14, expcnt / lgkmcnt at max)
template <int N>
DLTB_DEV void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

template <int D, int ROWS, bool ASM = false>
struct GldsTile {
  static constexpr int CH = D / 8;
  static constexpr int NI = ROWS * CH / 256;   // wave-instructions per wave (4 waves per tile)
  static_assert(ROWS * CH % 256 == 0, "tile must split into whole wave-instructions");
  DLTB_DEV static void load(const bf16_t* base, long stride, int row0, char* tile, int wv, int lane) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int lin = (wv * NI + i) * 64 + lane;
      const int row = lin / CH, pos = lin % CH;
      const bf16_t* src = base + (long)(row0 + row) * stride + ((pos ^ swz<D>(row)) << 3);
      if constexpr (ASM)
        glds16_asm(src, tile + (wv * NI + i) * 1024);
      else
        __builtin_amdgcn_global_load_lds((const void*)src,
                                         (__attribute__((address_space(3))) void*)(tile + (wv * NI + i) * 1024),
                                         16, 0, 0);
    }
  }
  // per-lane byte offsets of the NI DMA instructions relative to row row0 (tile-invariant)
  DLTB_DEV static void offsets(long stride, int wv, int lane, uint32_t (&off)[NI]) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int lin = (wv * NI + i) * 64 + lane;
      const int row = lin / CH, pos = lin % CH;
      off[i] = (uint32_t)((row * stride + ((pos ^ swz<D>(row)) << 3)) * 2);
    }
  }
  // rows row0 .. row0 + ROWS - 1 with row0 folded into the (wave-uniform) base pointer
  DLTB_DEV static void load_sv(const bf16_t* base_row0, const uint32_t (&off)[NI], char* tile, int wv) {
#pragma unroll
    for (int i = 0; i < NI; ++i) glds16_sv(base_row0, off[i], tile + (wv * NI + i) * 1024);
  }
};

}  // namespace
