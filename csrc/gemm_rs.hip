// bf16 "NT" GEMM with register-staged operands for the per-layer products of a training step
// (gfx950, CDNA4):
//
//   C[M, N] = A[M][K] . B[N][K]^T  (+ bias[n])  (+ C when accumulating)       fp32 accumulate
//
// Every forward product (x W^T) and every data gradient against the cached W^T of a TinyGPT /
// Mistral block has this form with M = tokens.  At M = 2048 the output of one product is only
// 2-8 M elements, so one tile per CU is all the parallelism there is; each CU then has to pull
// (BM + BN) x K x 2 bytes of operands through its 64 B/clk L2 -> CU path, and that stream -- not
// the MFMAs -- sets the floor of the N = 1024 products (docs: profiles/gemm_roofline_r5.txt).
//
// Design (round 5, replaces gemm_nt.hip's LDS-DMA loader/consumer split as the step's kernel):
//   * 256 threads = 4 waves, one workgroup per CU; every wave both loads and multiplies.
//   * Operands are staged global -> VGPRs -> LDS.  A plain global_load_dwordx4 costs its wave a
//     few issue cycles (an LDS-DMA instruction holds its wave ~60-100), so the loads of D stages
//     can be kept in flight in registers between the MFMAs of the current stage: per thread and
//     stage NA + NB 16-byte pieces, one 128-byte row segment per 8 consecutive lanes (full cache
//     lines), written to LDS with ds_write_b128 one stage before the MFMAs read it.
//   * Two LDS buffers, ONE barrier per 64-deep k-step: stage t+1 is written into the buffer that
//     the previous k-step read (all waves passed that step's barrier after draining their reads)
//     while the MFMAs of stage t read the other buffer.
//   * LDS image [row][64] bf16 with the 16-byte chunk XOR-swizzled by (row >> 1) & 7: conflict-free
//     for the ds_write_b128 groups (8 lanes = one row) and for the ds_read_b128 fragment groups of
//     both the 16x16x32 and the 32x32x16 MFMA (16 distinct rows per 16-lane group).
//   * MFMA operands swapped (B fragment as the MFMA's A operand), so a lane holds 4 consecutive
//     output columns of one row: 8-byte stores with the bias / accumulate fused in the epilogue.
//   * XCD-aware tile walk: workgroups b, b + 8, ... share an XCD under round-robin dispatch (speed
//     only); each XCD's tiles form a gm x (tiles / 8 / gm) block so its A and B panels are shared
//     in the XCD's 4 MB L2.
#include "common.h"
#include "launchers.h"

namespace {

typedef h16_t rs_frag __attribute__((ext_vector_type(8)));    // 8 x bf16: one MFMA A/B fragment
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // 16 bytes in 4 VGPRs
typedef __attribute__((address_space(3))) u32x4 lds_u4t;
typedef __attribute__((address_space(3))) f32x4 lds_f4t;

struct RsArgs {
  const bf16_t* a;
  const bf16_t* b;
  bf16_t* c;
  const bf16_t* bias;
  long lda, ldb, ldc;
  int M, N, K;
  int gm;            // m-tiles per group of the XCD-aware walk
  int accumulate;
  // fp32-image kernels only: C = (A B^T) * aux elementwise (aux [M, N] bf16, row stride ldc), rounded once, and
  // part[m-tile][n] = the column sums of the rounded C over the tile's rows (the dGELU epilogue: aux = GELU'(f))
  const bf16_t* aux;
  float* part;
  // fp32-image kernels only: gout = GELU(C) of the rounded C (row stride ldc) -- the fc1 forward's activation
  // written by the producing GEMM instead of a separate elementwise pass over f
  bf16_t* gout;
};

DLTB_DEV f32x4 mfma16(rs_frag a, rs_frag b, f32x4 c) {
#if DLTB_F16
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
#else
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
#endif
}
DLTB_DEV f32x16 mfma32(rs_frag a, rs_frag b, f32x16 c) {
#if DLTB_F16
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
#else
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
#endif
}

// Coalesced epilogue through LDS (the stage buffers are free after the k-loop's last barrier).  An MFMA
// accumulator gives each lane 4 consecutive columns of ONE row, so storing it directly is a row-per-lane
// store: every 8-byte store instruction touches 64 rows (cache lines) -- store-issue bound, ~2-9 us at the
// end of every product.  Phase 1: each lane adds the bias in fp32, rounds once to bf16 and writes its
// 8-byte pieces into a [BM][BN + 8] image (16-byte aligned rows, b64 writes conflict-free); phase 2: 16-byte
// chunks, 8 lanes per 128-byte row segment, to global memory (accumulate adds the old C there, in fp32).
template <int BM, int BN>
struct RsEpi {
  static constexpr int P = BN + 8;                 // row pitch (elements)
  static constexpr int BYTES = BM * P * 2;
  DLTB_DEV static void put(uint32_t lds0, const bf16_t* bias, int n0, int ml, int nl, const float* a) {
    float v[4] = {a[0], a[1], a[2], a[3]};
    if (bias) {
      const uint2 bb = *reinterpret_cast<const uint2*>(bias + n0 + nl);
      v[0] += lo_bf(bb.x); v[1] += hi_bf(bb.x); v[2] += lo_bf(bb.y); v[3] += hi_bf(bb.y);
    }
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 o = {pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
    *(__attribute__((address_space(3))) u32x2*)(size_t)(lds0 + (ml * P + nl) * 2) = o;
  }
  DLTB_DEV static void flush(const RsArgs& g, uint32_t lds0, int m0, int n0, int tid) {
    constexpr int CPR = BN / 8, CHUNKS = BM * CPR;
    static_assert(CHUNKS % 256 == 0, "epilogue chunks");
#pragma unroll 4
    for (int c = tid; c < CHUNKS; c += 256) {
      const int row = c / CPR, ch = c - row * CPR;
      u32x4 v = *(lds_u4t*)(size_t)(lds0 + (row * P + ch * 8) * 2);
      bf16_t* dst = g.c + (size_t)(m0 + row) * g.ldc + n0 + ch * 8;
      if (g.accumulate) {
        const u32x4 old = *reinterpret_cast<const u32x4*>(dst);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          v[e] = pack_bf2(lo_bf(v[e]) + lo_bf(old[e]), hi_bf(v[e]) + hi_bf(old[e]));
      }
      *reinterpret_cast<u32x4*>(dst) = v;
    }
  }
};

// fp32 variant (the 3-buffer kernels, whose stage buffers hold a [BM][BN + 4] fp32 image): phase 1 stores the
// raw accumulators (16-byte writes, 8 rows per lane group: conflict-free at the BN + 4 pitch); phase 2 adds the
// bias and rounds ONCE.  Phase 2 gives every thread 4 columns of a row (16-byte LDS read, 8-byte global store:
// a wave covers 256 contiguous columns).  When BN / 4 divides 256 a thread keeps the same 4 columns in every
// row it stores, so its bias is loaded once at kernel start (prefetched: no bias latency in the epilogue).
template <int BM, int BN, int NT = 256>
struct RsEpiF {
  static constexpr int P = BN + 4;                 // row pitch (fp32 elements)
  static constexpr int BYTES = BM * P * 4;
  static constexpr int CPR = BN / 4;               // 4-column chunks per row
  static constexpr bool FIXED = NT % CPR == 0;     // the thread's columns are the same in every row
  struct Bias {
    float v[4];
  };
  DLTB_DEV static Bias prefetch(const bf16_t* bias, int n0, int tid) {
    Bias b{{0.f, 0.f, 0.f, 0.f}};
    if (FIXED && bias) {
      const uint2 bb = *reinterpret_cast<const uint2*>(bias + n0 + (tid % CPR) * 4);
      b.v[0] = lo_bf(bb.x); b.v[1] = hi_bf(bb.x); b.v[2] = lo_bf(bb.y); b.v[3] = hi_bf(bb.y);
    }
    return b;
  }
  DLTB_DEV static void put(uint32_t lds0, int ml, int nl, const float* a) {
    *(lds_f4t*)(size_t)(lds0 + (ml * P + nl) * 4) = f32x4{a[0], a[1], a[2], a[3]};
  }
  // the aux values of this thread's epilogue chunks, loaded at kernel start (the aux operand is cold: its
  // loads issued in the epilogue exposed their HBM latency row after row)
  static constexpr int ITER = BM * CPR / NT;
  static constexpr bool AUX_PF = ITER <= 16;            // <= 32 VGPRs held through the k-loop
  struct Aux {
    uint2 v[AUX_PF ? ITER : 1];
  };
  DLTB_DEV static void prefetch_aux(const RsArgs& g, int m0, int n0, int tid, Aux& ax) {
    if constexpr (AUX_PF) {
      if (g.aux) {
#pragma unroll
        for (int i = 0; i < ITER; ++i) {
          const int c = tid + i * NT, row = c / CPR, ch = c - row * CPR;
          ax.v[i] = *reinterpret_cast<const uint2*>(g.aux + (size_t)(m0 + row) * g.ldc + n0 + ch * 4);
        }
      }
    }
  }
  DLTB_DEV static void flush(const RsArgs& g, uint32_t lds0, int m0, int n0, int tid, const Bias& pb,
                             const Aux& ax = Aux{}) {
    constexpr int CHUNKS = BM * CPR;
    static_assert(CHUNKS % NT == 0, "epilogue chunks");
    float cs[4] = {0.f, 0.f, 0.f, 0.f};                // dGELU epilogue: this thread's column sums
#pragma unroll
    for (int i = 0; i < ITER; ++i) {                   // fully unrolled: ax.v[i] stays in registers
      const int c = tid + i * NT;
      const int row = c / CPR, ch = c - row * CPR;
      const f32x4 x = *(lds_f4t*)(size_t)(lds0 + (row * P + ch * 4) * 4);
      float v[4] = {x[0], x[1], x[2], x[3]};
      if (FIXED) {
        v[0] += pb.v[0]; v[1] += pb.v[1]; v[2] += pb.v[2]; v[3] += pb.v[3];
      } else if (g.bias) {
        const uint2 bb = *reinterpret_cast<const uint2*>(g.bias + n0 + ch * 4);
        v[0] += lo_bf(bb.x); v[1] += hi_bf(bb.x); v[2] += lo_bf(bb.y); v[3] += hi_bf(bb.y);
      }
      const size_t off = (size_t)(m0 + row) * g.ldc + n0 + ch * 4;
      bf16_t* dst = g.c + off;
      if (g.accumulate) {
        const uint2 old = *reinterpret_cast<const uint2*>(dst);
        v[0] += lo_bf(old.x); v[1] += hi_bf(old.x); v[2] += lo_bf(old.y); v[3] += hi_bf(old.y);
      }
      if (g.aux) {
        uint2 a2;
        if constexpr (AUX_PF) a2 = ax.v[i];
        else a2 = *reinterpret_cast<const uint2*>(g.aux + off);
        v[0] *= lo_bf(a2.x); v[1] *= hi_bf(a2.x); v[2] *= lo_bf(a2.y); v[3] *= hi_bf(a2.y);
      }
      uint2 o;
      o.x = pack_bf2(v[0], v[1]);
      o.y = pack_bf2(v[2], v[3]);
      *reinterpret_cast<uint2*>(dst) = o;
      if (g.gout) {                                    // GELU of the stored (rounded) f, as gelu_fwd_kernel
        uint2 go;
        go.x = pack_bf2(gelu_fwd_f(lo_bf(o.x)), gelu_fwd_f(hi_bf(o.x)));
        go.y = pack_bf2(gelu_fwd_f(lo_bf(o.y)), gelu_fwd_f(hi_bf(o.y)));
        *reinterpret_cast<uint2*>(g.gout + off) = go;
      }
      if (g.part) {                                    // sum the rounded values the next GEMM reads
        cs[0] += lo_bf(o.x); cs[1] += hi_bf(o.x); cs[2] += lo_bf(o.y); cs[3] += hi_bf(o.y);
      }
    }
    if (FIXED && g.part) {
      // threads t, t + CPR, ... hold the same 4 columns: fold them through LDS (the image is free once
      // every thread has stored its rows), one partial row per m-tile
      constexpr int G = NT / CPR;
      __syncthreads();
      *(lds_f4t*)(size_t)(lds0 + tid * 16) = f32x4{cs[0], cs[1], cs[2], cs[3]};
      __syncthreads();
      if (tid < CPR) {
        f32x4 t = *(lds_f4t*)(size_t)(lds0 + tid * 16);
#pragma unroll
        for (int j = 1; j < G; ++j) t += *(lds_f4t*)(size_t)(lds0 + (tid + j * CPR) * 16);
        *reinterpret_cast<float4*>(g.part + (size_t)(m0 / BM) * g.N + n0 + tid * 4) = make_float4(t[0], t[1], t[2], t[3]);
      }
    }
  }
};

template <int BM, int BN, int WGM, int D, bool M32, int NW = 4>
struct RsGeo {
  static_assert(NW % WGM == 0, "wave grid");
  static constexpr int WGN = NW / WGM;
  static constexpr int PR = 8 * NW;                       // rows per staging pass (8 lanes per 128-byte row)
  static constexpr int PSTRIDE = PR * 128;                // LDS bytes per staging pass
  static constexpr int BK = 64;
  static constexpr int WM = BM / WGM, WN = BN / WGN;     // wave tile
  static constexpr int T = M32 ? 32 : 16;                 // MFMA output edge
  static constexpr int FM = WM / T, FN = WN / T;          // MFMA tiles per wave
  static constexpr int KS = M32 ? 4 : 2;                  // MFMA k-steps per 64-deep stage
  static constexpr int NA = BM / PR, NB = BN / PR;        // 16-byte pieces per thread per stage
  static constexpr int NI = NA + NB;
  static constexpr int A_BYTES = BM * 128, STAGE = (BM + BN) * 128;
  static constexpr int U = D % 2 == 0 ? D : 2 * D;        // k-loop unroll: register set and LDS buffer both static
  static constexpr int ACC = M32 ? 16 : 4;
  static_assert(WM % T == 0 && WN % T == 0 && BM % PR == 0 && BN % PR == 0, "tile shape");
};

// Workgroup barrier that no LDS access can cross in either direction.  __syncthreads() alone is not a
// compiler barrier for these accesses: hipcc (ROCm 7.2) sank a fragment read of the buffer that the
// next k-step overwrites below the barrier that was to order it -- other waves' writes then raced it
// (wrong tiles whenever waves drifted apart, e.g. with 2-3 workgroups per CU; scripts/debug_gemm_rs.py).
DLTB_DEV void rs_barrier() {
  asm volatile("" ::: "memory");
  __syncthreads();
  asm volatile("" ::: "memory");
}

DLTB_DEV uint32_t lane_addr(uint32_t sbase, uint32_t off) {
  uint32_t a;
  asm("v_add_u32 %0, %1, %2" : "=v"(a) : "s"(sbase), "v"(off));
  return a;
}

DLTB_DEV void wait_vm0() { __builtin_amdgcn_s_waitcnt((0) | (0 << 14) | (7 << 4) | (15 << 8)); }

// byte offset of 16-byte chunk `ch` of row `row` in a [rows][64] bf16 LDS image
DLTB_DEV uint32_t rs_off(int row, int ch) { return (uint32_t)(row * 128 + ((ch ^ ((row >> 1) & 7)) << 4)); }

template <int BM, int BN, int WGM, int D, bool M32, int DBG = 0>
__global__ __launch_bounds__(256, 1) void gemm_rs_kernel(RsArgs g) {
  using G = RsGeo<BM, BN, WGM, D, M32>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WGM, wn = wave / WGM;

  // ---- tile walk: XCD-major, then groups of gm m-tiles x all n-tiles
  const int tiles_n = g.N / BN, tiles_m = g.M / BM, tiles = tiles_m * tiles_n;
  const int L = blockIdx.x;
  int idx = L;
  if ((tiles & 7) == 0) idx = (L & 7) * (tiles >> 3) + (L >> 3);
  int mb, nb;
  if (g.gm > 1 && tiles_m % g.gm == 0) {
    const int span = g.gm * tiles_n, grp = idx / span, in = idx - grp * span;
    mb = grp * g.gm + in % g.gm;
    nb = in / g.gm;
  } else {
    mb = idx / tiles_n;
    nb = idx - mb * tiles_n;
  }
  const int m0 = mb * BM, n0 = nb * BN;
  const int nk = g.K / G::BK;
  DLTB_DCHECK(m0 + BM <= g.M && n0 + BN <= g.N && nk * G::BK == g.K && nk % G::U == 0);

  // ---- staging addresses: piece i of a thread = row 32 i + tid / 8, chunk tid % 8 of the tile
  const int prow = tid >> 3, pch = tid & 7;
  const char* abase = (const char*)(g.a + (long)m0 * g.lda);   // wave-uniform
  const char* bbase = (const char*)(g.b + (long)n0 * g.ldb);
  uint32_t voa[G::NA], vob[G::NB];
#pragma unroll
  for (int i = 0; i < G::NA; ++i) voa[i] = (uint32_t)(((32 * i + prow) * g.lda + pch * 8) * 2);
#pragma unroll
  for (int i = 0; i < G::NB; ++i) vob[i] = (uint32_t)(((32 * i + prow) * g.ldb + pch * 8) * 2);
  const uint32_t wlane = rs_off(prow, pch);   // + 4096 i: rows 32 i + prow keep the swizzle of prow
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) char*)smem;

  u32x4 R[D][G::NI];
  auto gload = [&](int kt, u32x4 (&r)[G::NI]) {
    const int ks = min(kt, nk - 1) * (G::BK * 2);    // past the end: re-read the last stage (never written to a live buffer)
    const char* pa = abase + ks;
    const char* pb = bbase + ks;
#pragma unroll
    for (int i = 0; i < G::NA; ++i) r[i] = *reinterpret_cast<const u32x4*>(pa + voa[i]);
#pragma unroll
    for (int i = 0; i < G::NB; ++i) r[G::NA + i] = *reinterpret_cast<const u32x4*>(pb + vob[i]);
  };
  auto swrite = [&](int buf, const u32x4 (&r)[G::NI]) {
    const uint32_t base = lds0 + buf * G::STAGE + wlane;
#pragma unroll
    for (int i = 0; i < G::NA; ++i) *(lds_u4t*)(size_t)(base + 4096 * i) = r[i];
#pragma unroll
    for (int i = 0; i < G::NB; ++i) *(lds_u4t*)(size_t)(base + G::A_BYTES + 4096 * i) = r[G::NA + i];
  };

  // ---- fragment read offsets (lane part; the row base of each fragment is an immediate)
  // 16x16x32: lane l reads row (l & 15), chunk 4 kk + (l >> 4);  32x32x16: row (l & 31), chunk 2 s + (l >> 5)
  constexpr int RL = M32 ? 32 : 16;
  const int fr = lane & (RL - 1), fq = M32 ? (lane >> 5) : (lane >> 4);
  uint32_t foff[G::KS];
#pragma unroll
  for (int s = 0; s < G::KS; ++s) foff[s] = rs_off(fr, (M32 ? 2 : 4) * s + fq);
  const int arow0 = wm * G::WM, brow0 = wn * G::WN;

  using Acc = typename std::conditional<M32, f32x16, f32x4>::type;
  Acc acc[G::FM][G::FN];
#pragma unroll
  for (int i = 0; i < G::FM; ++i)
#pragma unroll
    for (int j = 0; j < G::FN; ++j) acc[i][j] = Acc{};

  // A k-step's MFMAs in two halves (k 0-31 / 32-63 of the stage), each with its own fragment set
  // X / Y, so the reads of the next half overlap the MFMAs of the current one.
  constexpr int KH = G::KS / 2;
  struct Frags {
    rs_frag a[KH][G::FM], b[KH][G::FN];
  };
  auto fread = [&](Frags& f, int buf, int half) {
    const uint32_t base = lds0 + buf * G::STAGE;
#pragma unroll
    for (int s = 0; s < KH; ++s) {
#pragma unroll
      for (int i = 0; i < G::FM; ++i)
        f.a[s][i] = __builtin_bit_cast(
            rs_frag, *(lds_u4t*)(size_t)(base + foff[half * KH + s] + (arow0 + G::T * i) * 128));
#pragma unroll
      for (int j = 0; j < G::FN; ++j)
        f.b[s][j] = __builtin_bit_cast(
            rs_frag, *(lds_u4t*)(size_t)(base + G::A_BYTES + foff[half * KH + s] + (brow0 + G::T * j) * 128));
    }
  };
  auto mma = [&](const Frags& f) {
    if constexpr ((DBG & 8) != 0) {          // ablation: operands kept live, no MFMA
#pragma unroll
      for (int s = 0; s < KH; ++s) {
#pragma unroll
        for (int i = 0; i < G::FM; ++i) asm volatile("" ::"v"(f.a[s][i]));
#pragma unroll
        for (int j = 0; j < G::FN; ++j) asm volatile("" ::"v"(f.b[s][j]));
      }
      return;
    }
#pragma unroll
    for (int s = 0; s < KH; ++s)
#pragma unroll
      for (int i = 0; i < G::FM; ++i)
#pragma unroll
        for (int j = 0; j < G::FN; ++j) {
          if constexpr (M32) acc[i][j] = mfma32(f.b[s][j], f.a[s][i], acc[i][j]);
          else acc[i][j] = mfma16(f.b[s][j], f.a[s][i], acc[i][j]);
        }
  };

  // ---- prologue: D stages in flight; stages 0 and 1 in LDS buffers 0 / 1, stage 0's fragments in X / Y
  Frags X, Y;
#pragma unroll
  for (int d = 0; d < D; ++d) gload(d, R[d]);
  swrite(0, R[0]);
  gload(D, R[0]);
  rs_barrier();                                      // stage 0 visible
  fread(X, 0, 0);
  swrite(1, R[1 % D]);
  gload(D + 1, R[1 % D]);
  fread(Y, 0, 1);
  rs_barrier();                                      // stage 1 visible, stage 0's reads drained

  // ---- main loop.  Top of k-step kt: X / Y hold stage kt's fragments, stage kt + 1 is visible in
  // buffer (kt + 1) & 1 and buffer kt & 1 is free (every wave drained its reads of stage kt before
  // the barrier); R[(kt + 2) % D] holds stage kt + 2.  Segment: MFMAs of half 0 while the next
  // stage's half-0 fragments are read and stage kt + 2 is written into the free buffer (its
  // registers re-issued for stage kt + 2 + D), then MFMAs of half 1 while the half-1 fragments are
  // read; one barrier.  (Past the end the reads fetch unused data and the writes re-store the last
  // stage into a buffer nobody reads again.)
  for (int t = 0; t < nk; t += G::U) {
#pragma unroll
    for (int u = 0; u < G::U; ++u) {
      const int kt = t + u;
      // (DBG & 16 / 32 / 64: ablation builds without the loop's global loads / fragment reads and
      // MFMAs / LDS writes -- timing only)
      if constexpr ((DBG & 32) == 0) mma(X);
      if constexpr ((DBG & 4) != 0) rs_barrier();
      if constexpr ((DBG & 32) == 0) fread(X, (u + 1) & 1, 0);
      if constexpr ((DBG & 64) == 0) swrite(u & 1, R[(u + 2) % D]);
      if constexpr ((DBG & 16) == 0) gload(kt + 2 + D, R[(u + 2) % D]);
      if constexpr ((DBG & 32) == 0) mma(Y);
      if constexpr ((DBG & 4) != 0) rs_barrier();
      if constexpr ((DBG & 32) == 0) fread(Y, (u + 1) & 1, 1);
      rs_barrier();
    }
  }
  if constexpr ((DBG & 1) != 0) wait_vm0();

  // ---- epilogue: lane -> row m, 4 consecutive columns per register group, through LDS
  using E = RsEpi<BM, BN>;
  static_assert(E::BYTES <= 2 * G::STAGE, "epilogue image exceeds the stage buffers");
#pragma unroll
  for (int i = 0; i < G::FM; ++i) {
#pragma unroll
    for (int j = 0; j < G::FN; ++j) {
#pragma unroll
      for (int q = 0; q < G::ACC / 4; ++q) {
        // 16x16: columns 4 fq .. +3;  32x32: register group q -> columns 8 q + 4 fq .. +3
        const float a4[4] = {acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
        E::put(lds0, g.bias, n0, arow0 + G::T * i + fr, brow0 + G::T * j + (M32 ? 8 * q + 4 * fq : 4 * fq), a4);
      }
    }
  }
  rs_barrier();
  E::flush(g, lds0, m0, n0, tid);
}

// ---------------------------------------------------------------------------------------------------
// Software-pipelined variant (round 5, the step's kernel): three LDS buffers and an explicit instruction
// interleave.  hipcc emits a k-step's MFMAs as one back-to-back cluster; a wave alone on its SIMD issues in
// order, so the LDS reads, LDS writes and global loads queued behind that cluster only start when its last
// MFMA has issued, and the MFMA pipe then idles while they drain (ablation: MFMA time and memory time
// ADD UP -- cfg 16-25).  Here each k-step is two halves and every MFMA of a half is followed by its share
// of the memory instructions (__builtin_amdgcn_sched_group_barrier), so they issue in the MFMA shadows:
//   segment kt (stage s lives in LDS buffer s % 3):
//     MFMAs of half 0 (X)  ||  read half 1 of stage kt into Y, write stage kt + 2, load stage kt + 2 + D
//     MFMAs of half 1 (Y)  ||  read half 0 of stage kt + 1 into X
//     one barrier
// Buffer (kt + 2) % 3 held stage kt - 1, whose last reads were issued before the previous barrier; the
// reads of stage kt / kt + 1 are of stages written two / one segments earlier.  Global loads are buffer
// loads (the k offset in the SGPR soffset: no per-load address VALU).
template <int N>
struct RsInt {
  // distribute T items over N slots: the count of slot k
  static constexpr int share(int T, int k) { return (T * (k + 1)) / N - (T * k) / N; }
};
template <int NM, int NR, int NW, int NL, int K = 0>
DLTB_DEV void rs_interleave() {
  if constexpr (K < NM) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                           // one MFMA
    constexpr int r = RsInt<NM>::share(NR, K), w = RsInt<NM>::share(NW, K), l = RsInt<NM>::share(NL, K);
    if constexpr (r > 0) __builtin_amdgcn_sched_group_barrier(0x100, r, 0);       // DS reads
    if constexpr (w > 0) __builtin_amdgcn_sched_group_barrier(0x200, w, 0);       // DS writes
    if constexpr (l > 0) __builtin_amdgcn_sched_group_barrier(0x020, l, 0);       // VMEM reads
    rs_interleave<NM, NR, NW, NL, K + 1>();
  }
}

template <int BM, int BN, int WGM, int D, bool M32>
__global__ __launch_bounds__(256, 1) void gemm_rsp_kernel(RsArgs g) {
  using G = RsGeo<BM, BN, WGM, D, M32>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WGM, wn = wave / WGM;

  const int tiles_n = g.N / BN, tiles_m = g.M / BM, tiles = tiles_m * tiles_n;
  const int L = blockIdx.x;
  int idx = L;
  if ((tiles & 7) == 0) idx = (L & 7) * (tiles >> 3) + (L >> 3);
  int mb, nb;
  if (g.gm > 1 && tiles_m % g.gm == 0) {
    const int span = g.gm * tiles_n, grp = idx / span, in = idx - grp * span;
    mb = grp * g.gm + in % g.gm;
    nb = in / g.gm;
  } else {
    mb = idx / tiles_n;
    nb = idx - mb * tiles_n;
  }
  const int m0 = mb * BM, n0 = nb * BN;
  const int nk = g.K / G::BK;
  DLTB_DCHECK(m0 + BM <= g.M && n0 + BN <= g.N && nk * G::BK == g.K && nk % D == 0 && nk >= 2);

  const int prow = tid >> 3, pch = tid & 7;
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)(g.a + (long)m0 * g.lda), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc((void*)(g.b + (long)n0 * g.ldb), (short)0, 0x7fffffff, 0x00020000);
  uint32_t voa[G::NA], vob[G::NB];
#pragma unroll
  for (int i = 0; i < G::NA; ++i) voa[i] = (uint32_t)(((32 * i + prow) * g.lda + pch * 8) * 2);
#pragma unroll
  for (int i = 0; i < G::NB; ++i) vob[i] = (uint32_t)(((32 * i + prow) * g.ldb + pch * 8) * 2);
  const uint32_t wlane = rs_off(prow, pch);
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) char*)smem;

  u32x4 R[D][G::NI];
  auto gload = [&](int kt, u32x4 (&r)[G::NI]) {
    const int so = min(kt, nk - 1) * (G::BK * 2);   // past the end: the last stage again (never consumed)
#pragma unroll
    for (int i = 0; i < G::NA; ++i) r[i] = __builtin_amdgcn_raw_buffer_load_b128(ra, voa[i], so, 0);
#pragma unroll
    for (int i = 0; i < G::NB; ++i) r[G::NA + i] = __builtin_amdgcn_raw_buffer_load_b128(rb, vob[i], so, 0);
  };
  auto swrite = [&](uint32_t bufbase, const u32x4 (&r)[G::NI]) {
    const uint32_t base = bufbase + wlane;
#pragma unroll
    for (int i = 0; i < G::NA; ++i) *(lds_u4t*)(size_t)(base + 4096 * i) = r[i];
#pragma unroll
    for (int i = 0; i < G::NB; ++i) *(lds_u4t*)(size_t)(base + G::A_BYTES + 4096 * i) = r[G::NA + i];
  };

  constexpr int RL = M32 ? 32 : 16;
  const int fr = lane & (RL - 1), fq = M32 ? (lane >> 5) : (lane >> 4);
  const int arow0 = wm * G::WM, brow0 = wn * G::WN;
  // per-lane fragment offsets with the wave's row base folded in: a fragment read is then one
  // (buffer base + lane offset) add per k-substep and operand, the tile rows an immediate offset
  uint32_t foa[G::KS], fob[G::KS];
#pragma unroll
  for (int s = 0; s < G::KS; ++s) {
    foa[s] = rs_off(fr, (M32 ? 2 : 4) * s + fq) + arow0 * 128;
    fob[s] = rs_off(fr, (M32 ? 2 : 4) * s + fq) + G::A_BYTES + brow0 * 128;
  }

  using Acc = typename std::conditional<M32, f32x16, f32x4>::type;
  Acc acc[G::FM][G::FN];
#pragma unroll
  for (int i = 0; i < G::FM; ++i)
#pragma unroll
    for (int j = 0; j < G::FN; ++j) acc[i][j] = Acc{};

  constexpr int KH = G::KS / 2;
  struct Frags {
    rs_frag a[KH][G::FM], b[KH][G::FN];
  };
  auto fread = [&](Frags& f, uint32_t bufbase, int half) {
#pragma unroll
    for (int s = 0; s < KH; ++s) {
      const uint32_t pa = lane_addr(bufbase, foa[half * KH + s]), pb = lane_addr(bufbase, fob[half * KH + s]);
#pragma unroll
      for (int i = 0; i < G::FM; ++i)
        f.a[s][i] = __builtin_bit_cast(rs_frag, *(lds_u4t*)(size_t)(pa + G::T * i * 128));
#pragma unroll
      for (int j = 0; j < G::FN; ++j)
        f.b[s][j] = __builtin_bit_cast(rs_frag, *(lds_u4t*)(size_t)(pb + G::T * j * 128));
    }
  };
  auto mma = [&](const Frags& f) {
#pragma unroll
    for (int s = 0; s < KH; ++s)
#pragma unroll
      for (int i = 0; i < G::FM; ++i)
#pragma unroll
        for (int j = 0; j < G::FN; ++j) {
          if constexpr (M32) acc[i][j] = mfma32(f.b[s][j], f.a[s][i], acc[i][j]);
          else acc[i][j] = mfma16(f.b[s][j], f.a[s][i], acc[i][j]);
        }
  };
  constexpr int NM = KH * G::FM * G::FN, NR = KH * (G::FM + G::FN);

  // ---- prologue: stages 0 and 1 in buffers 0 / 1, half 0 of stage 0 in X
  Frags X, Y;
#pragma unroll
  for (int d = 0; d < D; ++d) gload(d, R[d]);
  swrite(lds0, R[0]);
  gload(D, R[0]);
  swrite(lds0 + G::STAGE, R[1 % D]);
  gload(D + 1, R[1 % D]);
  rs_barrier();
  fread(X, lds0, 0);
  uint32_t b_cur = lds0, b_nxt = lds0 + G::STAGE, b_wr = lds0 + 2 * G::STAGE;   // stage kt, kt + 1, kt + 2

  for (int t = 0; t < nk; t += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int kt = t + u;
      mma(X);
      fread(Y, b_cur, 1);
      swrite(b_wr, R[(u + 2) % D]);
      gload(kt + 2 + D, R[(u + 2) % D]);
      rs_interleave<NM, NR, G::NI, G::NI>();
      mma(Y);
      fread(X, b_nxt, 0);
      rs_interleave<NM, NR, 0, 0>();
      rs_barrier();
      const uint32_t b_old = b_cur;
      b_cur = b_nxt;
      b_nxt = b_wr;
      b_wr = b_old;
    }
  }

  using E = RsEpi<BM, BN>;
  static_assert(E::BYTES <= 3 * G::STAGE, "epilogue image exceeds the stage buffers");
#pragma unroll
  for (int i = 0; i < G::FM; ++i) {
#pragma unroll
    for (int j = 0; j < G::FN; ++j) {
#pragma unroll
      for (int q = 0; q < G::ACC / 4; ++q) {
        const float a4[4] = {acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
        E::put(lds0, g.bias, n0, arow0 + G::T * i + fr, brow0 + G::T * j + (M32 ? 8 * q + 4 * fq : 4 * fq), a4);
      }
    }
  }
  rs_barrier();
  E::flush(g, lds0, m0, n0, tid);
}

template <int BM, int BN, int WGM, int D, bool M32>
void launch_rsp(const RsArgs& g, hipStream_t st) {
  constexpr int smem = 3 * RsGeo<BM, BN, WGM, D, M32>::STAGE;
  static_assert(smem <= 163840, "LDS budget");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_rsp_kernel<BM, BN, WGM, D, M32>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  const int tiles = (g.M / BM) * (g.N / BN);
  hipLaunchKernelGGL((gemm_rsp_kernel<BM, BN, WGM, D, M32>), dim3(tiles), dim3(256), smem, st, g);
}

// ---------------------------------------------------------------------------------------------------
// Fenced schedule (kind 3): the rsp pipeline with the issue order written out and pinned.  In the rsp build
// hipcc honoured the sched_group_barrier masks only in part -- MFMAs of the second half were pulled into
// the first half's slots, the fragment reads they need were queued right in front of them
// (s_waitcnt lgkmcnt(0) before every few MFMAs) and the LDS writes + global loads issued as one cluster.
// Here every MFMA is followed by its slot of memory instructions, with a full scheduling fence
// (__builtin_amdgcn_sched_barrier(0)) around each slot, so the program order IS the issue order:
//   half 0: MFMA q of stage kt (X), then Y-read / LDS-write / global-load share q     (q < NM)
//   half 1: MFMA q of stage kt (Y), then X-read share q (half 0 of stage kt + 1)
//   s_waitcnt lgkmcnt(NR) (this segment's LDS writes done, the X reads may stay in flight) + s_barrier
// LDS operations complete in order, so the waits the compiler places before each MFMA are partial.
template <int BM, int BN, int WGM, int D, bool M32, int DBG = 0, int NW = 4>
__global__ __launch_bounds__(64 * NW, 1) void gemm_rsf_kernel(RsArgs g) {
  using G = RsGeo<BM, BN, WGM, D, M32, NW>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WGM, wn = wave / WGM;

  const int tiles_n = g.N / BN, tiles_m = g.M / BM, tiles = tiles_m * tiles_n;
  const int L = blockIdx.x;
  int idx = L;
  if ((tiles & 7) == 0) idx = (L & 7) * (tiles >> 3) + (L >> 3);
  int mb, nb;
  if (g.gm > 1 && tiles_m % g.gm == 0) {
    const int span = g.gm * tiles_n, grp = idx / span, in = idx - grp * span;
    mb = grp * g.gm + in % g.gm;
    nb = in / g.gm;
  } else {
    mb = idx / tiles_n;
    nb = idx - mb * tiles_n;
  }
  const int m0 = mb * BM, n0 = nb * BN;
  const int nk = g.K / G::BK;
  DLTB_DCHECK(m0 + BM <= g.M && n0 + BN <= g.N && nk * G::BK == g.K && nk % D == 0 && nk >= 2);

  const int prow = tid >> 3, pch = tid & 7;
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)(g.a + (long)m0 * g.lda), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc((void*)(g.b + (long)n0 * g.ldb), (short)0, 0x7fffffff, 0x00020000);
  uint32_t voa[G::NA], vob[G::NB];
#pragma unroll
  for (int i = 0; i < G::NA; ++i) voa[i] = (uint32_t)(((G::PR * i + prow) * g.lda + pch * 8) * 2);
#pragma unroll
  for (int i = 0; i < G::NB; ++i) vob[i] = (uint32_t)(((G::PR * i + prow) * g.ldb + pch * 8) * 2);
  const uint32_t wlane = rs_off(prow, pch);
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) char*)smem;
  using E = RsEpiF<BM, BN, 64 * NW>;
  const typename E::Bias pbias = E::prefetch(g.bias, n0, tid);
  typename E::Aux paux;
  E::prefetch_aux(g, m0, n0, tid, paux);

  constexpr int RL = M32 ? 32 : 16;
  const int fr = lane & (RL - 1), fq = M32 ? (lane >> 5) : (lane >> 4);
  const int arow0 = wm * G::WM, brow0 = wn * G::WN;
  uint32_t foa[G::KS], fob[G::KS];
#pragma unroll
  for (int s = 0; s < G::KS; ++s) {
    foa[s] = rs_off(fr, (M32 ? 2 : 4) * s + fq) + arow0 * 128;
    fob[s] = rs_off(fr, (M32 ? 2 : 4) * s + fq) + G::A_BYTES + brow0 * 128;
  }

  using Acc = typename std::conditional<M32, f32x16, f32x4>::type;
  Acc acc[G::FM][G::FN];
#pragma unroll
  for (int i = 0; i < G::FM; ++i)
#pragma unroll
    for (int j = 0; j < G::FN; ++j) acc[i][j] = Acc{};

  constexpr int KH = G::KS / 2;
  constexpr int FPS = G::FM + G::FN;                    // fragments per k-substep
  constexpr int NM = KH * G::FM * G::FN, NR = KH * FPS;
  static_assert(NR <= 15, "lgkmcnt field");
  struct Frags {
    rs_frag f[KH][FPS];                                  // a fragments, then b fragments
  };
  u32x4 R[D][G::NI];

  // single memory operations, by index (all indices compile-time after unrolling)
  auto read1 = [&](Frags& F, uint32_t bufbase, int half, int r) {
    const int s = r / FPS, f = r - s * FPS;
    const uint32_t off = f < G::FM ? foa[half * KH + s] + G::T * f * 128
                                   : fob[half * KH + s] + G::T * (f - G::FM) * 128;
    F.f[s][f] = __builtin_bit_cast(rs_frag, *(lds_u4t*)(size_t)(bufbase + off));
  };
  auto write1 = [&](uint32_t bufbase, const u32x4 (&r)[G::NI], int w) {
    const uint32_t off = w < G::NA ? G::PSTRIDE * w : G::A_BYTES + G::PSTRIDE * (w - G::NA);
    *(lds_u4t*)(size_t)(bufbase + wlane + off) = r[w];
  };
  auto load1 = [&](int kt, u32x4 (&r)[G::NI], int l) {
    const int so = min(kt, nk - 1) * (G::BK * 2);
    if (l < G::NA) r[l] = __builtin_amdgcn_raw_buffer_load_b128(ra, voa[l], so, 0);
    else r[l] = __builtin_amdgcn_raw_buffer_load_b128(rb, vob[l - G::NA], so, 0);
  };
  auto mma1 = [&](const Frags& F, int q) {
    const int s = q / (G::FM * G::FN), i = (q / G::FN) % G::FM, j = q % G::FN;
    if constexpr (M32) acc[i][j] = mfma32(F.f[s][G::FM + j], F.f[s][i], acc[i][j]);
    else acc[i][j] = mfma16(F.f[s][G::FM + j], F.f[s][i], acc[i][j]);
  };

  auto keepall = [&](const Frags& F) {
#pragma unroll
    for (int s = 0; s < KH; ++s)
#pragma unroll
      for (int f = 0; f < FPS; ++f) asm volatile("" ::"v"(F.f[s][f]));
  };
  auto keep1 = [&](const Frags& F, int q) {           // ablation: the operands of MFMA q stay live
    const int s = q / (G::FM * G::FN), i = (q / G::FN) % G::FM, j = q % G::FN;
    asm volatile("" ::"v"(F.f[s][i]), "v"(F.f[s][G::FM + j]));
  };

  Frags X, Y;
#pragma unroll
  for (int d = 0; d < D; ++d)
#pragma unroll
    for (int l = 0; l < G::NI; ++l) load1(d, R[d], l);
#pragma unroll
  for (int w = 0; w < G::NI; ++w) write1(lds0, R[0], w);
#pragma unroll
  for (int l = 0; l < G::NI; ++l) load1(D, R[0], l);
#pragma unroll
  for (int w = 0; w < G::NI; ++w) write1(lds0 + G::STAGE, R[1 % D], w);
#pragma unroll
  for (int l = 0; l < G::NI; ++l) load1(D + 1, R[1 % D], l);
  rs_barrier();
#pragma unroll
  for (int r = 0; r < NR; ++r) read1(X, lds0, 0, r);
  uint32_t b_cur = lds0, b_nxt = lds0 + G::STAGE, b_wr = lds0 + 2 * G::STAGE;

  for (int t = 0; t < nk; t += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int kt = t + u;
      u32x4 (&RR)[G::NI] = R[(u + 2) % D];
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < NM; ++q) {
        // (DBG & 8 / 16 / 32 / 64: timing-only ablations without fragment reads / loop global loads /
        // MFMAs / LDS writes)
        if constexpr ((DBG & 32) == 0) mma1(X, q);
        else keep1(X, q);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int r = (NR * q) / NM; r < (NR * (q + 1)) / NM; ++r)
          if constexpr ((DBG & 8) == 0) read1(Y, b_cur, 1, r);
#pragma unroll
        for (int w = (G::NI * q) / NM; w < (G::NI * (q + 1)) / NM; ++w) {
          if constexpr ((DBG & 64) == 0) write1(b_wr, RR, w);
          else asm volatile("" ::"v"(RR[w]));
          if constexpr ((DBG & 16) == 0) load1(kt + 2 + D, RR, w);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      // DBG & 128: every X fragment stays live to the end of its half, so the Y reads issued between the X
      // MFMAs cannot be given the registers of a fragment an MFMA in flight is still reading (the register
      // allocator otherwise reuses each fragment's registers right after its last MFMA)
      if constexpr ((DBG & 128) != 0) keepall(X);
#pragma unroll
      for (int q = 0; q < NM; ++q) {
        if constexpr ((DBG & 32) == 0) mma1(Y, q);
        else keep1(Y, q);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int r = (NR * q) / NM; r < (NR * (q + 1)) / NM; ++r)
          if constexpr ((DBG & 8) == 0) read1(X, b_nxt, 0, r);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr ((DBG & 128) != 0) keepall(Y);          // (see the X half)
      // this segment's LDS writes complete (the NR X reads issued after them may still be in flight:
      // they read b_nxt, which nobody writes before the NEXT barrier), then the workgroup barrier
      asm volatile("s_waitcnt lgkmcnt(%0)\n\ts_barrier" ::"n"(NR) : "memory");
      __builtin_amdgcn_sched_barrier(0);
      const uint32_t b_old = b_cur;
      b_cur = b_nxt;
      b_nxt = b_wr;
      b_wr = b_old;
    }
  }

  rs_barrier();                                          // all fragment reads done before the epilogue image
  static_assert(E::BYTES <= 3 * G::STAGE, "epilogue image exceeds the stage buffers");
#pragma unroll
  for (int i = 0; i < G::FM; ++i) {
#pragma unroll
    for (int j = 0; j < G::FN; ++j) {
#pragma unroll
      for (int q = 0; q < G::ACC / 4; ++q) {
        const float a4[4] = {acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
        E::put(lds0, arow0 + G::T * i + fr, brow0 + G::T * j + (M32 ? 8 * q + 4 * fq : 4 * fq), a4);
      }
    }
  }
  rs_barrier();
  E::flush(g, lds0, m0, n0, tid, pbias, paux);
}

template <int BM, int BN, int WGM, int D, bool M32, int DBG = 0, int NW = 4>
void launch_rsf(const RsArgs& g, hipStream_t st) {
  constexpr int smem = 3 * RsGeo<BM, BN, WGM, D, M32, NW>::STAGE;
  static_assert(smem <= 163840, "LDS budget");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_rsf_kernel<BM, BN, WGM, D, M32, DBG, NW>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  const int tiles = (g.M / BM) * (g.N / BN);
  hipLaunchKernelGGL((gemm_rsf_kernel<BM, BN, WGM, D, M32, DBG, NW>), dim3(tiles), dim3(64 * NW), smem, st, g);
}

// ---------------------------------------------------------------------------------------------------
// Direct-operand variant: the four waves split ONE operand's rows (PA: A / M, else B / N), so each wave's
// rows of that operand are private -- they are loaded straight into MFMA fragments (16 rows x 64
// contiguous bytes per load instruction, natural 16x16x32 k order), with no LDS round trip; only the
// other operand, which all four waves read, is staged through LDS.  Per 64-deep k-step of a 128 x 64 tile
// with A direct: 8 KB of ds_write and 32 KB of ds_read instead of 24 + 48 KB, and 8 ds_read_b128 per wave
// instead of 12.  DP stages of private fragments and DS stages of the shared operand are in flight.
template <int BM, int BN, bool PA, int DP, int DS>
struct RsdGeo {
  static constexpr int P_ROWS = PA ? BM : BN, S_ROWS = PA ? BN : BM;
  static constexpr int PW = P_ROWS / 4;                 // private rows per wave
  static constexpr int FP = PW / 16, FS = S_ROWS / 16;   // 16x16 MFMA tiles per wave along P / S
  static constexpr int NS = S_ROWS / 32;                 // 16-byte pieces per thread per stage (shared operand)
  static constexpr int STAGE = S_ROWS * 128;
  static constexpr int U = (DP > DS ? DP : DS) < 2 ? 2 : (DP > DS ? DP : DS);   // DP, DS in {1, 2, 4}
  static_assert(PW % 16 == 0 && S_ROWS % 32 == 0 && U % DP == 0 && U % DS == 0 && U % 2 == 0, "geometry");
};

template <int BM, int BN, bool PA, int DP, int DS>
__global__ __launch_bounds__(256, 1) void gemm_rsd_kernel(RsArgs g) {
  using G = RsdGeo<BM, BN, PA, DP, DS>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  const int tiles_n = g.N / BN, tiles_m = g.M / BM, tiles = tiles_m * tiles_n;
  const int L = blockIdx.x;
  int idx = L;
  if ((tiles & 7) == 0) idx = (L & 7) * (tiles >> 3) + (L >> 3);
  int mb, nb;
  if (g.gm > 1 && tiles_m % g.gm == 0) {
    const int span = g.gm * tiles_n, grp = idx / span, in = idx - grp * span;
    mb = grp * g.gm + in % g.gm;
    nb = in / g.gm;
  } else {
    mb = idx / tiles_n;
    nb = idx - mb * tiles_n;
  }
  const int m0 = mb * BM, n0 = nb * BN;
  const int nk = g.K / 64;
  DLTB_DCHECK(m0 + BM <= g.M && n0 + BN <= g.N && nk * 64 == g.K && nk % G::U == 0);

  const long pld = PA ? g.lda : g.ldb, sld = PA ? g.ldb : g.lda;
  const char* pbase = PA ? (const char*)(g.a + (long)m0 * g.lda) : (const char*)(g.b + (long)n0 * g.ldb);
  const char* sbase = PA ? (const char*)(g.b + (long)n0 * g.ldb) : (const char*)(g.a + (long)m0 * g.lda);
  const int fr = lane & 15, fq = lane >> 4;
  // private fragment i of a wave: rows wave * PW + 16 i + fr, bytes 64 kk + 16 fq of the stage's 128
  uint32_t vp[G::FP];
#pragma unroll
  for (int i = 0; i < G::FP; ++i) vp[i] = (uint32_t)(((wave * G::PW + 16 * i + fr) * pld) * 2 + 16 * fq);
  // shared operand staging: piece i of a thread = row 32 i + tid / 8, chunk tid % 8
  const int prow = tid >> 3, pch = tid & 7;
  uint32_t vs[G::NS];
#pragma unroll
  for (int i = 0; i < G::NS; ++i) vs[i] = (uint32_t)(((32 * i + prow) * sld + pch * 8) * 2);
  const uint32_t wlane = rs_off(prow, pch);
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) char*)smem;
  uint32_t foff[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) foff[kk] = rs_off(fr, 4 * kk + fq);

  struct PFrag {
    rs_frag f[G::FP][2];
  };
  PFrag PR[DP];
  u32x4 R[DS][G::NS];
  auto pload = [&](int kt, PFrag& d) {
    const char* pp = pbase + min(kt, nk - 1) * 128;
#pragma unroll
    for (int i = 0; i < G::FP; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        d.f[i][kk] = __builtin_bit_cast(rs_frag, *reinterpret_cast<const u32x4*>(pp + vp[i] + 64 * kk));
  };
  auto sload = [&](int kt, u32x4 (&r)[G::NS]) {
    const char* ps = sbase + min(kt, nk - 1) * 128;
#pragma unroll
    for (int i = 0; i < G::NS; ++i) r[i] = *reinterpret_cast<const u32x4*>(ps + vs[i]);
  };
  auto swrite = [&](int buf, const u32x4 (&r)[G::NS]) {
    const uint32_t base = lds0 + buf * G::STAGE + wlane;
#pragma unroll
    for (int i = 0; i < G::NS; ++i) *(lds_u4t*)(size_t)(base + 4096 * i) = r[i];
  };
  struct SFrag {
    rs_frag f[G::FS];
  };
  auto fread = [&](SFrag& x, int buf, int kk) {
    const uint32_t base = lds0 + buf * G::STAGE + foff[kk];
#pragma unroll
    for (int j = 0; j < G::FS; ++j) x.f[j] = __builtin_bit_cast(rs_frag, *(lds_u4t*)(size_t)(base + 16 * j * 128));
  };
  f32x4 acc[G::FP][G::FS];
#pragma unroll
  for (int i = 0; i < G::FP; ++i)
#pragma unroll
    for (int j = 0; j < G::FS; ++j) acc[i][j] = f32x4{};
  // MFMA(B fragment, A fragment): lane -> m, registers -> 4 consecutive n
  auto mma = [&](const PFrag& p, int kk, const SFrag& x) {
#pragma unroll
    for (int i = 0; i < G::FP; ++i)
#pragma unroll
      for (int j = 0; j < G::FS; ++j) {
        if constexpr (PA) acc[i][j] = mfma16(x.f[j], p.f[i][kk], acc[i][j]);
        else acc[i][j] = mfma16(p.f[i][kk], x.f[j], acc[i][j]);
      }
  };

  SFrag X, Y;
#pragma unroll
  for (int d = 0; d < DP; ++d) pload(d, PR[d]);
#pragma unroll
  for (int d = 0; d < DS; ++d) sload(d, R[d]);
  swrite(0, R[0]);
  sload(DS, R[0]);
  rs_barrier();
  fread(X, 0, 0);
  swrite(1, R[1 % DS]);
  sload(DS + 1, R[1 % DS]);
  fread(Y, 0, 1);
  rs_barrier();
  for (int t = 0; t < nk; t += G::U) {
#pragma unroll
    for (int u = 0; u < G::U; ++u) {
      const int kt = t + u;
      mma(PR[u % DP], 0, X);
      fread(X, (u + 1) & 1, 0);
      swrite(u & 1, R[(u + 2) % DS]);
      sload(kt + 2 + DS, R[(u + 2) % DS]);
      mma(PR[u % DP], 1, Y);
      fread(Y, (u + 1) & 1, 1);
      pload(kt + DP, PR[u % DP]);
      rs_barrier();
    }
  }

  using E = RsEpi<BM, BN>;
#pragma unroll
  for (int i = 0; i < G::FP; ++i) {
#pragma unroll
    for (int j = 0; j < G::FS; ++j) {
      const int ml = PA ? wave * G::PW + 16 * i + fr : 16 * j + fr;
      const int nl = PA ? 16 * j + 4 * fq : wave * G::PW + 16 * i + 4 * fq;
      const float a4[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      E::put(lds0, g.bias, n0, ml, nl, a4);
    }
  }
  rs_barrier();
  E::flush(g, lds0, m0, n0, tid);
}

template <int BM, int BN, bool PA, int DP, int DS>
void launch_rsd(const RsArgs& g, hipStream_t st) {
  constexpr int ring = 2 * RsdGeo<BM, BN, PA, DP, DS>::STAGE, epi = RsEpi<BM, BN>::BYTES;
  constexpr int smem = ring > epi ? ring : epi;
  static_assert(smem <= 163840, "LDS budget");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_rsd_kernel<BM, BN, PA, DP, DS>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  const int tiles = (g.M / BM) * (g.N / BN);
  hipLaunchKernelGGL((gemm_rsd_kernel<BM, BN, PA, DP, DS>), dim3(tiles), dim3(256), smem, st, g);
}

// ---------------------------------------------------------------------------------------------------
// Fenced direct-operand kernel (kind 4).  Ablations of the fenced kernel (profiles/gemm_rs_instep_ab_r5.txt) put
// the LDS at the top of the per-k-step budget: every staged byte crosses the VGPR -> LDS store path (~79 B/clk per
// CU) once and the fragment reads twice.  Here the four waves split ONE operand's rows (PA: A / the tile's M, else
// B / N), so each wave's rows of that operand are private to it and go global -> VGPR straight in MFMA fragment
// order, never touching the LDS; only the other ("shared") operand is staged through the three LDS buffers.  At
// 128 x 64 with A private the LDS carries 8 KB of stores and 32 KB of fragment reads per 64-deep k-step instead of
// 24 + 48 KB.
// k order: a 32x32x16 fragment holds, in lane l, 8 consecutive k of row (l & 31) from k-half h = l >> 5.  The
// k-chunk (8 elements) that MFMA substep s takes from half h is chunk 4 h + s of the 64-deep stage -- a
// permutation of the stage's k applied to BOTH operands alike (the product is unchanged), chosen so that a lane's
// four private fragments of a stage are 64 contiguous bytes of its row: 4 buffer loads at offsets 0/16/32/48.
// Private stages: D register sets; stage kt + D's substeps 0-1 are loaded in segment kt's second half (after the
// MFMAs that last read that set's substeps 0-1), substeps 2-3 in segment kt + 1's first half.
template <int BM, int BN, bool PA, int D>
struct RsgGeo {
  static constexpr int P_ROWS = PA ? BM : BN, S_ROWS = PA ? BN : BM;
  static constexpr int PW = P_ROWS / 4;              // private rows per wave
  static constexpr int FP = PW / 32, FS = S_ROWS / 32;
  static constexpr int NS = S_ROWS / 32;             // shared 16-byte pieces per thread per stage
  static constexpr int STAGE = S_ROWS * 128;
  static_assert(PW % 32 == 0 && S_ROWS % 32 == 0, "tile shape");
};

template <int BM, int BN, bool PA, int D>
__global__ __launch_bounds__(256, 1) void gemm_rsg_kernel(RsArgs g) {
  using G = RsgGeo<BM, BN, PA, D>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  const int tiles_n = g.N / BN, tiles_m = g.M / BM, tiles = tiles_m * tiles_n;
  const int L = blockIdx.x;
  int idx = L;
  if ((tiles & 7) == 0) idx = (L & 7) * (tiles >> 3) + (L >> 3);
  int mb, nb;
  if (g.gm > 1 && tiles_m % g.gm == 0) {
    const int span = g.gm * tiles_n, grp = idx / span, in = idx - grp * span;
    mb = grp * g.gm + in % g.gm;
    nb = in / g.gm;
  } else {
    mb = idx / tiles_n;
    nb = idx - mb * tiles_n;
  }
  const int m0 = mb * BM, n0 = nb * BN;
  const int nk = g.K / 64;
  DLTB_DCHECK(m0 + BM <= g.M && n0 + BN <= g.N && nk * 64 == g.K && nk % D == 0 && nk >= 2);

  const bf16_t* pbase = PA ? g.a + (long)m0 * g.lda : g.b + (long)n0 * g.ldb;
  const bf16_t* sbase = PA ? g.b + (long)n0 * g.ldb : g.a + (long)m0 * g.lda;
  const long pld = PA ? g.lda : g.ldb, sld = PA ? g.ldb : g.lda;
  const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc((void*)pbase, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsh = __builtin_amdgcn_make_buffer_rsrc((void*)sbase, (short)0, 0x7fffffff, 0x00020000);
  const int fr = lane & 31, fh = lane >> 5;
  uint32_t vop[G::FP];                                  // private: row (wave rows + 32 i + fr), k-half fh
#pragma unroll
  for (int i = 0; i < G::FP; ++i) vop[i] = (uint32_t)(((wave * G::PW + 32 * i + fr) * pld) * 2 + fh * 64);
  const int prow = tid >> 3, pch = tid & 7;
  uint32_t vos[G::NS];                                  // shared staging: row 32 i + tid / 8, chunk tid % 8
#pragma unroll
  for (int i = 0; i < G::NS; ++i) vos[i] = (uint32_t)(((32 * i + prow) * sld + pch * 8) * 2);
  const uint32_t wlane = rs_off(prow, pch);
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) char*)smem;
  const typename RsEpiF<BM, BN>::Bias pbias = RsEpiF<BM, BN>::prefetch(g.bias, n0, tid);
  uint32_t fos[4];                                      // shared fragment: row fr, chunk 4 fh + s
#pragma unroll
  for (int s = 0; s < 4; ++s) fos[s] = rs_off(fr, 4 * fh + s);

  f32x16 acc[G::FP][G::FS];
#pragma unroll
  for (int i = 0; i < G::FP; ++i)
#pragma unroll
    for (int j = 0; j < G::FS; ++j) acc[i][j] = f32x16{};

  rs_frag P[D][4][G::FP];                               // private fragments: stage set, substep, row block
  u32x4 R[D][G::NS];                                    // shared staging registers
  struct Half {
    rs_frag f[2][G::FS];                                // shared fragments of two substeps
  };
  constexpr int NR = 2 * G::FS;                         // shared fragment reads per half
  static_assert(NR <= 15, "lgkmcnt field");

  auto pload1 = [&](int kt, rs_frag (&p)[4][G::FP], int s, int i) {
    const int so = min(kt, nk - 1) * 128 + 16 * s;
    p[s][i] = __builtin_bit_cast(rs_frag, __builtin_amdgcn_raw_buffer_load_b128(rp, vop[i], so, 0));
  };
  auto sload1 = [&](int kt, u32x4 (&r)[G::NS], int l) {
    r[l] = __builtin_amdgcn_raw_buffer_load_b128(rsh, vos[l], min(kt, nk - 1) * 128, 0);
  };
  auto swrite1 = [&](uint32_t bufbase, const u32x4 (&r)[G::NS], int w) {
    *(lds_u4t*)(size_t)(bufbase + wlane + 4096 * w) = r[w];
  };
  auto sread1 = [&](Half& H, uint32_t bufbase, int half, int r) {
    const int s = r / G::FS, j = r - s * G::FS;
    H.f[s][j] = __builtin_bit_cast(rs_frag, *(lds_u4t*)(size_t)(bufbase + fos[2 * half + s] + 32 * j * 128));
  };
  auto mma1 = [&](const Half& H, const rs_frag (&p)[4][G::FP], int half, int q) {
    const int s = q / (G::FP * G::FS), i = (q / G::FS) % G::FP, j = q % G::FS;
    // D[n][m]: the MFMA's A operand is the B-matrix fragment (lane = n), its B operand the A-matrix one
    if constexpr (PA) acc[i][j] = mfma32(H.f[s][j], p[2 * half + s][i], acc[i][j]);
    else acc[i][j] = mfma32(p[2 * half + s][i], H.f[s][j], acc[i][j]);
  };
  constexpr int NM = 2 * G::FP * G::FS;                 // MFMAs per half
  constexpr int NPL = 2 * G::FP;                        // private loads per half (two substeps)

  // prologue: private stages 0 .. D-1 and shared stages 0 .. D-1 in flight, shared stages 0 / 1 in buffers 0 / 1
  Half X, Y;
#pragma unroll
  for (int d = 0; d < D; ++d) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < G::FP; ++i) pload1(d, P[d], s, i);
#pragma unroll
    for (int l = 0; l < G::NS; ++l) sload1(d, R[d], l);
  }
#pragma unroll
  for (int w = 0; w < G::NS; ++w) swrite1(lds0, R[0], w);
#pragma unroll
  for (int l = 0; l < G::NS; ++l) sload1(D, R[0], l);
#pragma unroll
  for (int w = 0; w < G::NS; ++w) swrite1(lds0 + G::STAGE, R[1 % D], w);
#pragma unroll
  for (int l = 0; l < G::NS; ++l) sload1(D + 1, R[1 % D], l);
  rs_barrier();
#pragma unroll
  for (int r = 0; r < NR; ++r) sread1(X, lds0, 0, r);
  uint32_t b_cur = lds0, b_nxt = lds0 + G::STAGE, b_wr = lds0 + 2 * G::STAGE;

  for (int t = 0; t < nk; t += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int kt = t + u;
      rs_frag (&PC)[4][G::FP] = P[u];                   // this stage's private fragments
      rs_frag (&PPrev)[4][G::FP] = P[(u + D - 1) % D];  // stage kt - 1's set: its substeps 2-3 reload now
      u32x4 (&RR)[G::NS] = R[(u + 2) % D];
      __builtin_amdgcn_sched_barrier(0);
      // half 0: MFMAs of substeps 0-1 || shared reads of substeps 2-3, shared write / load, private loads
      // of stage kt - 1 + D substeps 2-3 (their set was last read by segment kt - 1's second half)
#pragma unroll
      for (int q = 0; q < NM; ++q) {
        mma1(X, PC, 0, q);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int r = (NR * q) / NM; r < (NR * (q + 1)) / NM; ++r) sread1(Y, b_cur, 1, r);
#pragma unroll
        for (int w = (G::NS * q) / NM; w < (G::NS * (q + 1)) / NM; ++w) {
          swrite1(b_wr, RR, w);
          sload1(kt + 2 + D, RR, w);
        }
#pragma unroll
        for (int l = (NPL * q) / NM; l < (NPL * (q + 1)) / NM; ++l)   // (kt = 0: stage D - 1 again, same data)
          pload1(kt - 1 + D, PPrev, 2 + l / G::FP, l % G::FP);
        __builtin_amdgcn_sched_barrier(0);
      }
      // half 1: MFMAs of substeps 2-3 || shared reads of the next stage's substeps 0-1, private loads of
      // stage kt + D substeps 0-1 into this stage's set
#pragma unroll
      for (int q = 0; q < NM; ++q) {
        mma1(Y, PC, 1, q);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int r = (NR * q) / NM; r < (NR * (q + 1)) / NM; ++r) sread1(X, b_nxt, 0, r);
#pragma unroll
        for (int l = (NPL * q) / NM; l < (NPL * (q + 1)) / NM; ++l) pload1(kt + D, PC, l / G::FP, l % G::FP);
        __builtin_amdgcn_sched_barrier(0);
      }
      asm volatile("s_waitcnt lgkmcnt(%0)\n\ts_barrier" ::"n"(NR) : "memory");
      __builtin_amdgcn_sched_barrier(0);
      const uint32_t b_old = b_cur;
      b_cur = b_nxt;
      b_nxt = b_wr;
      b_wr = b_old;
    }
  }

  rs_barrier();
  using E = RsEpiF<BM, BN>;
  static_assert(E::BYTES <= 163840, "epilogue image exceeds the LDS");
#pragma unroll
  for (int i = 0; i < G::FP; ++i) {
#pragma unroll
    for (int j = 0; j < G::FS; ++j) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float a4[4] = {acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
        // lane: column m = fr of its MFMA tile, rows n = 8 q + 4 fh .. + 3
        const int pr = wave * G::PW + 32 * i, sr = 32 * j;
        if constexpr (PA) E::put(lds0, pr + fr, sr + 8 * q + 4 * fh, a4);
        else E::put(lds0, sr + fr, pr + 8 * q + 4 * fh, a4);
      }
    }
  }
  rs_barrier();
  E::flush(g, lds0, m0, n0, tid, pbias);
}

template <int BM, int BN, bool PA, int D>
void launch_rsg(const RsArgs& g, hipStream_t st) {
  constexpr int st3 = 3 * RsgGeo<BM, BN, PA, D>::STAGE, epi = RsEpiF<BM, BN>::BYTES;
  constexpr int smem = st3 > epi ? st3 : epi;
  static_assert(smem <= 163840, "LDS budget");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_rsg_kernel<BM, BN, PA, D>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  const int tiles = (g.M / BM) * (g.N / BN);
  hipLaunchKernelGGL((gemm_rsg_kernel<BM, BN, PA, D>), dim3(tiles), dim3(256), smem, st, g);
}

template <int BM, int BN, int WGM, int D, bool M32, int DBG = 0>
void launch_rs(const RsArgs& g, hipStream_t st) {
  // (DBG & 2: debug builds pad the LDS to 100 KB: one workgroup per CU)
  constexpr int smem = 2 * RsGeo<BM, BN, WGM, D, M32>::STAGE + ((DBG & 2) ? 102400 : 0);
  static_assert(smem <= 163840, "LDS budget");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_rs_kernel<BM, BN, WGM, D, M32, DBG>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  const int tiles = (g.M / BM) * (g.N / BN);
  hipLaunchKernelGGL((gemm_rs_kernel<BM, BN, WGM, D, M32, DBG>), dim3(tiles), dim3(256), smem, st, g);
}

struct RsCfg {
  int bm, bn, wgm, d;
  bool m32;
  int dp = 0;        // > 0: direct-operand kernel, DP stages of private fragments (d = shared stages)
  bool pa = false;   // direct kernel: A private (waves split M), else B private (waves split N)
  int kind = 0;      // 2: software-pipelined kernel (3 LDS buffers), 3: same with a fenced schedule
};
// 0-2: N = 1024 products (16 x 16 tiles of 128 x 64); 3-4 / 6: N = 4096 (128 x 256); 5: N = 3072 (128 x 192);
// 8-12: direct-operand kernels
constexpr RsCfg kRsCfgs[] = {{128, 64, 2, 2, false}, {128, 64, 2, 4, false}, {128, 64, 2, 2, true},
                             {128, 256, 2, 2, false}, {128, 256, 2, 2, true}, {128, 192, 2, 2, false},
                             {128, 128, 2, 2, false}, {64, 128, 2, 2, false},
                             {128, 64, 4, 2, false, 2, true}, {128, 64, 4, 2, false, 4, true},
                             {128, 256, 1, 2, false, 2, false}, {128, 192, 1, 2, false, 2, false},
                             {128, 128, 4, 2, false, 2, true},
                             // 13-15: debug variants of cfg 0 (vmcnt(0) before the epilogue / one workgroup
                             // per CU / a barrier after every MFMA half)
                             {128, 64, 2, 2, false}, {128, 64, 2, 2, false}, {128, 64, 2, 2, false},
                             // 16-19 / 20-23: ablations of cfg 4 / cfg 1 (no MFMA / no loop loads / no
                             // fragment reads + MFMA / no LDS writes): timing only
                             {128, 256, 2, 2, true}, {128, 256, 2, 2, true}, {128, 256, 2, 2, true},
                             {128, 256, 2, 2, true}, {128, 64, 2, 4, false}, {128, 64, 2, 4, false},
                             {128, 64, 2, 4, false}, {128, 64, 2, 4, false},
                             // 24 / 25: cfg 4 / cfg 1 with an empty k-loop (launch + prologue + epilogue)
                             {128, 256, 2, 2, true}, {128, 64, 2, 4, false},
                             // 26-31: software-pipelined kernel (gemm_rsp_kernel; kind 2)
                             {128, 64, 2, 2, false, 0, false, 2}, {128, 64, 2, 4, false, 0, false, 2},
                             {128, 64, 2, 4, true, 0, false, 2}, {128, 256, 2, 2, true, 0, false, 2},
                             {128, 192, 2, 2, false, 0, false, 2}, {128, 128, 2, 2, true, 0, false, 2},
                             // 32-37: fenced schedule (gemm_rsf_kernel; kind 3), the shapes of 26-31
                             {128, 64, 2, 2, false, 0, false, 3}, {128, 64, 2, 4, false, 0, false, 3},
                             {128, 64, 2, 4, true, 0, false, 3}, {128, 256, 2, 2, true, 0, false, 3},
                             {128, 192, 2, 2, false, 0, false, 3}, {128, 128, 2, 2, true, 0, false, 3},
                             // 38-42: ablations of cfg 35 (no fragment reads / no loop loads / no MFMA /
                             // no LDS writes / nothing but the barriers) -- timing only; 43: cfg 35 at D 3
                             {128, 256, 2, 2, true, 0, false, 3}, {128, 256, 2, 2, true, 0, false, 3},
                             {128, 256, 2, 2, true, 0, false, 3}, {128, 256, 2, 2, true, 0, false, 3},
                             {128, 256, 2, 2, true, 0, false, 3}, {128, 256, 2, 3, true, 0, false, 3},
                             // 44-48: ablations of cfg 34 (as 38-42); 49: cfg 34 at D 2; 50: cfg 34 with the
                             // waves split 4 x 1 (32 x 64 each); 51: D 8
                             {128, 64, 2, 4, true, 0, false, 3}, {128, 64, 2, 4, true, 0, false, 3},
                             {128, 64, 2, 4, true, 0, false, 3}, {128, 64, 2, 4, true, 0, false, 3},
                             {128, 64, 2, 4, true, 0, false, 3}, {128, 64, 2, 2, true, 0, false, 3},
                             {128, 64, 4, 4, true, 0, false, 3}, {128, 64, 2, 8, true, 0, false, 3},
                             // 52-58: fenced direct-operand kernel (gemm_rsg_kernel; kind 4): 128 x 64 A private
                             // at D 4 / 2 / 8, 128 x 256 B private at D 2 / 4, 128 x 192 A private at D 2 / 4
                             {128, 64, 0, 4, true, 4, true, 4}, {128, 64, 0, 2, true, 2, true, 4},
                             {128, 64, 0, 8, true, 8, true, 4}, {128, 256, 0, 2, true, 2, false, 4},
                             {128, 256, 0, 4, true, 4, false, 4}, {128, 192, 0, 2, true, 2, true, 4},
                             {128, 192, 0, 4, true, 4, true, 4},
                             // 59-61: cfgs 35 / 34 / 36 with the fragment sets kept apart (DBG 128)
                             {128, 256, 2, 2, true, 0, false, 3}, {128, 64, 2, 4, true, 0, false, 3},
                             {128, 192, 2, 2, false, 0, false, 3},
                             // 62-66: fenced kernel with 8 waves (2 per SIMD: one wave's memory issue overlaps the
                             // other's MFMAs): 128 x 256 as 2 x 4 / 4 x 2 waves, 128 x 192 (16x16), 128 x 64 (32x32 /
                             // 16x16, 4 x 2 waves)
                             {128, 256, 2, 2, true, 0, false, 3}, {128, 256, 4, 2, true, 0, false, 3},
                             {128, 192, 2, 2, false, 0, false, 3}, {128, 64, 4, 4, true, 0, false, 3},
                             {128, 64, 4, 4, false, 0, false, 3},
                             // 67-69: 8-wave kernels at other depths: 128 x 256 D 4, 128 x 192 D 4, 128 x 64 D 2
                             {128, 256, 2, 4, true, 0, false, 3}, {128, 192, 2, 4, false, 0, false, 3},
                             {128, 64, 4, 2, true, 0, false, 3}};
constexpr int kRsNumCfgs = sizeof(kRsCfgs) / sizeof(kRsCfgs[0]);

void launch_rs_cfg(int cfg, const RsArgs& g, hipStream_t st) {
  switch (cfg) {
    case 0: launch_rs<128, 64, 2, 2, false>(g, st); break;
    case 1: launch_rs<128, 64, 2, 4, false>(g, st); break;
    case 2: launch_rs<128, 64, 2, 2, true>(g, st); break;
    case 3: launch_rs<128, 256, 2, 2, false>(g, st); break;
    case 4: launch_rs<128, 256, 2, 2, true>(g, st); break;
    case 5: launch_rs<128, 192, 2, 2, false>(g, st); break;
    case 6: launch_rs<128, 128, 2, 2, false>(g, st); break;
    case 7: launch_rs<64, 128, 2, 2, false>(g, st); break;
    case 8: launch_rsd<128, 64, true, 2, 2>(g, st); break;
    case 9: launch_rsd<128, 64, true, 4, 2>(g, st); break;
    case 10: launch_rsd<128, 256, false, 2, 2>(g, st); break;
    case 11: launch_rsd<128, 192, false, 2, 2>(g, st); break;
    case 12: launch_rsd<128, 128, true, 2, 2>(g, st); break;
    case 13: launch_rs<128, 64, 2, 2, false, 1>(g, st); break;
    case 14: launch_rs<128, 64, 2, 2, false, 2>(g, st); break;
    case 15: launch_rs<128, 64, 2, 2, false, 4>(g, st); break;
    case 16: launch_rs<128, 256, 2, 2, true, 8>(g, st); break;
    case 17: launch_rs<128, 256, 2, 2, true, 16>(g, st); break;
    case 18: launch_rs<128, 256, 2, 2, true, 32>(g, st); break;
    case 19: launch_rs<128, 256, 2, 2, true, 64>(g, st); break;
    case 20: launch_rs<128, 64, 2, 4, false, 8>(g, st); break;
    case 21: launch_rs<128, 64, 2, 4, false, 16>(g, st); break;
    case 22: launch_rs<128, 64, 2, 4, false, 32>(g, st); break;
    case 23: launch_rs<128, 64, 2, 4, false, 64>(g, st); break;
    case 24: launch_rs<128, 256, 2, 2, true, 112>(g, st); break;
    case 25: launch_rs<128, 64, 2, 4, false, 112>(g, st); break;
    case 26: launch_rsp<128, 64, 2, 2, false>(g, st); break;
    case 27: launch_rsp<128, 64, 2, 4, false>(g, st); break;
    case 28: launch_rsp<128, 64, 2, 4, true>(g, st); break;
    case 29: launch_rsp<128, 256, 2, 2, true>(g, st); break;
    case 30: launch_rsp<128, 192, 2, 2, false>(g, st); break;
    case 31: launch_rsp<128, 128, 2, 2, true>(g, st); break;
    case 32: launch_rsf<128, 64, 2, 2, false>(g, st); break;
    case 33: launch_rsf<128, 64, 2, 4, false>(g, st); break;
    case 34: launch_rsf<128, 64, 2, 4, true>(g, st); break;
    case 35: launch_rsf<128, 256, 2, 2, true>(g, st); break;
    case 36: launch_rsf<128, 192, 2, 2, false>(g, st); break;
    case 37: launch_rsf<128, 128, 2, 2, true>(g, st); break;
    case 38: launch_rsf<128, 256, 2, 2, true, 8>(g, st); break;
    case 39: launch_rsf<128, 256, 2, 2, true, 16>(g, st); break;
    case 40: launch_rsf<128, 256, 2, 2, true, 32>(g, st); break;
    case 41: launch_rsf<128, 256, 2, 2, true, 64>(g, st); break;
    case 42: launch_rsf<128, 256, 2, 2, true, 120>(g, st); break;
    case 43: launch_rsf<128, 256, 2, 3, true>(g, st); break;
    case 44: launch_rsf<128, 64, 2, 4, true, 8>(g, st); break;
    case 45: launch_rsf<128, 64, 2, 4, true, 16>(g, st); break;
    case 46: launch_rsf<128, 64, 2, 4, true, 32>(g, st); break;
    case 47: launch_rsf<128, 64, 2, 4, true, 64>(g, st); break;
    case 48: launch_rsf<128, 64, 2, 4, true, 120>(g, st); break;
    case 49: launch_rsf<128, 64, 2, 2, true>(g, st); break;
    case 50: launch_rsf<128, 64, 4, 4, true>(g, st); break;
    case 51: launch_rsf<128, 64, 2, 8, true>(g, st); break;
    case 52: launch_rsg<128, 64, true, 4>(g, st); break;
    case 53: launch_rsg<128, 64, true, 2>(g, st); break;
    case 54: launch_rsg<128, 64, true, 8>(g, st); break;
    case 55: launch_rsg<128, 256, false, 2>(g, st); break;
    case 56: launch_rsg<128, 256, false, 4>(g, st); break;
    case 57: launch_rsg<128, 192, true, 2>(g, st); break;
    case 58: launch_rsg<128, 192, true, 4>(g, st); break;
    case 59: launch_rsf<128, 256, 2, 2, true, 128>(g, st); break;
    case 60: launch_rsf<128, 64, 2, 4, true, 128>(g, st); break;
    case 61: launch_rsf<128, 192, 2, 2, false, 128>(g, st); break;
    case 62: launch_rsf<128, 256, 2, 2, true, 0, 8>(g, st); break;
    case 63: launch_rsf<128, 256, 4, 2, true, 0, 8>(g, st); break;
    case 64: launch_rsf<128, 192, 2, 2, false, 0, 8>(g, st); break;
    case 65: launch_rsf<128, 64, 4, 4, true, 0, 8>(g, st); break;
    case 66: launch_rsf<128, 64, 4, 4, false, 0, 8>(g, st); break;
    case 67: launch_rsf<128, 256, 2, 4, true, 0, 8>(g, st); break;
    case 68: launch_rsf<128, 192, 2, 4, false, 0, 8>(g, st); break;
    default: launch_rsf<128, 64, 4, 2, true, 0, 8>(g, st); break;
  }
}

}  // namespace

static bool rs_fits(int c, int M, int N, int K) {
  if (c < 0 || c >= kRsNumCfgs) return false;
  const RsCfg t = kRsCfgs[c];
  const int dm = t.dp > t.d ? t.dp : t.d;
  const int u = t.kind >= 2 ? t.d : t.dp > 0 ? (dm < 2 ? 2 : dm) : (t.d % 2 == 0 ? t.d : 2 * t.d);
  return M > 0 && N > 0 && K > 0 && M % t.bm == 0 && N % t.bn == 0 && K % 64 == 0 && (K / 64) % u == 0;
}

int dltb_gemm_rs_pick(int M, int N, int K) {
  // the config whose tile count is closest to one workgroup per CU (256); ties keep the earlier
  int best = -1, bestd = 1 << 30;
  for (int c = 0; c < kRsNumCfgs; ++c) {
    if (!rs_fits(c, M, N, K)) continue;
    const int tiles = (M / kRsCfgs[c].bm) * (N / kRsCfgs[c].bn);
    const int d = tiles > 256 ? (tiles - 256) * 2 : 256 - tiles;
    if (d < bestd) {
      bestd = d;
      best = c;
    }
  }
  return best;
}

bool dltb_gemm_rs_supported(int M, int N, int K, int cfg) {
  if (cfg < 0) cfg = dltb_gemm_rs_pick(M, N, K);
  return rs_fits(cfg, M, N, K);
}

int dltb_gemm_rs_bm(int cfg) { return (cfg >= 0 && cfg < kRsNumCfgs) ? kRsCfgs[cfg].bm : 0; }

bool dltb_gemm_rs_aux_supported(int M, int N, int K, int cfg) {
  // the aux / column-partial epilogue: fp32-image kernels (kinds 3), a thread's columns fixed across rows
  if (!dltb_gemm_rs_supported(M, N, K, cfg) || kRsCfgs[cfg].kind != 3) return false;
  const int nt = (cfg >= 62 && cfg <= 69) ? 512 : 256;
  const int cpr = kRsCfgs[cfg].bn / 4;
  return nt % cpr == 0 && kRsCfgs[cfg].bm * cpr / nt <= 16;   // the aux values prefetched (RsEpiF::AUX_PF)
}

bool dltb_gemm_rs_gelu_supported(int M, int N, int K, int cfg) {
  // the GELU-output epilogue: any fp32-image kernel (kind 3)
  if (cfg < 0) cfg = dltb_gemm_rs_pick(M, N, K);
  return dltb_gemm_rs_supported(M, N, K, cfg) && kRsCfgs[cfg].kind == 3;
}

int dltb_gemm_rs(const void* a, const void* b, void* c, const void* bias, long lda, long ldb, long ldc, int M,
                 int N, int K, int accumulate, int cfg, int gm, hipStream_t st, const void* aux, float* part,
                 void* gout) {
  if (cfg < 0) cfg = dltb_gemm_rs_pick(M, N, K);
  if (!dltb_gemm_rs_supported(M, N, K, cfg)) return -1;
  RsArgs g{};
  g.a = (const bf16_t*)a;
  g.b = (const bf16_t*)b;
  g.c = (bf16_t*)c;
  g.bias = (const bf16_t*)bias;
  g.lda = lda;
  g.ldb = ldb;
  g.ldc = ldc;
  g.M = M;
  g.N = N;
  g.K = K;
  g.gm = gm;
  g.accumulate = accumulate;
  g.aux = (const bf16_t*)aux;
  g.part = part;
  g.gout = (bf16_t*)gout;
  if ((aux || part) && !dltb_gemm_rs_aux_supported(M, N, K, cfg)) return -1;
  if (gout && (accumulate || !dltb_gemm_rs_gelu_supported(M, N, K, cfg))) return -1;
  launch_rs_cfg(cfg, g, st);
  return cfg;
}
