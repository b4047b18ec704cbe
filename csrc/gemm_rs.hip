// bf16 "NT" GEMM with register-staged operands for the per-layer products of a training step
// (gfx950, CDNA4):
//
//   C[M, N] = A[M][K] . B[N][K]^T  (+ bias[n])  (+ C when accumulating)       fp32 accumulate
//
// Every forward product (x W^T) and every data gradient against the cached W^T of a TinyGPT /
// Mistral block has this form with M = tokens.  At M = 2048 the output of one product is only
// 2-8 M elements, so one tile per CU is all the parallelism there is; each CU then has to pull
// (BM + BN) x K x 2 bytes of operands through its L2 -> CU path and round-trip them through LDS
// (docs: profiles/gemm_roofline_r5.txt).
//
// Design:
//   * one workgroup per CU; every wave both loads and multiplies.
//   * Operands are staged global -> VGPRs -> LDS.  A plain buffer_load_dwordx4 costs its wave a few
//     issue cycles (an LDS-DMA instruction holds its wave ~60-100), so the loads of D stages can be
//     kept in flight in registers between the MFMAs of the current stage: per thread and stage NA + NB
//     16-byte pieces, one 128-byte row segment per 8 consecutive lanes (full cache lines), written to
//     LDS with ds_write_b128 two stages before the MFMAs read it (three LDS buffers).
//   * LDS image [row][64] bf16 with the 16-byte chunk XOR-swizzled by (row >> 1) & 7: conflict-free
//     for the ds_write_b128 groups (8 lanes = one row) and for the ds_read_b128 fragment groups of
//     both the 16x16x32 and the 32x32x16 MFMA (16 distinct rows per 16-lane group).
//   * MFMA operands swapped (B fragment as the MFMA's A operand), so a lane holds 4 consecutive
//     output columns of one row; the fp32 tile goes through an LDS image to 8-byte stores with the
//     bias (prefetched at kernel start) / accumulate / GELU / dGELU epilogues fused.
//   * XCD-aware tile walk (below).
//   * optional K-split into two wave groups sharing the tile (gemm_rsf_kernel, KG = 2).
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

// Epilogue through an fp32 [BM][BN + 4] LDS image in the (free) stage buffers: phase 1 stores the
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
  DLTB_DEV static f32x4 get(uint32_t lds0, int ml, int nl) { return *(lds_f4t*)(size_t)(lds0 + (ml * P + nl) * 4); }
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

// byte offset of 16-byte chunk `ch` of row `row` in a [rows][64] bf16 LDS image
DLTB_DEV uint32_t rs_off(int row, int ch) { return (uint32_t)(row * 128 + ((ch ^ ((row >> 1) & 7)) << 4)); }

// ---------------------------------------------------------------------------------------------------
// The kernel: three LDS buffers per k-group and a fenced, software-pipelined issue order.  hipcc emits a
// k-step's MFMAs as one back-to-back cluster; a wave alone on its SIMD issues in order, so the LDS reads,
// LDS writes and global loads queued behind that cluster would only start when its last MFMA has issued
// (round-5 ablation: MFMA time and memory time ADD UP).  Here every MFMA is followed by its share of the
// memory instructions, with a full scheduling fence (__builtin_amdgcn_sched_barrier(0)) around each slot,
// so the program order IS the issue order:
//   segment j (stage s of the group lives in its LDS buffer s % 3):
//     half 0: MFMA q of stage j (fragments X), then Y-read / LDS-write / global-load share q   (q < NM)
//     half 1: MFMA q of stage j (fragments Y), then X-read share q (half 0 of stage j + 1)
//     s_waitcnt lgkmcnt(NR) (this segment's LDS writes done, the X reads may stay in flight) + s_barrier
// LDS operations complete in order, so the waits the compiler places before each MFMA are partial.
// Buffer (j + 2) % 3 held stage j - 1, whose last reads were issued before the previous barrier.
//
// K-split groups (KG = 2, round 6): the workgroup is two groups of NW waves that compute the SAME
// output tile over alternate 64-deep k-steps (group g: k-steps g, g + 2, ...), each with its own three
// stage buffers and registers, so every SIMD holds one wave of each group: while one wave waits on its
// LDS reads / writes or its loads, the other's MFMAs issue (unlike the 8-wave output split, each wave
// still reads only its own tile's fragments once per k-step).  The two fp32 partial tiles are summed once
// through the epilogue's LDS image.  STAG = 1 adds a barrier between the two halves of every segment and
// starts group 1 one barrier late, so each SIMD pairs one group's first half with the other's second half
// (MI355X_MICROARCH.md "two waves per SIMD", item 9: a half-block stagger).
template <int BM, int BN, int WGM, int D, bool M32, int NW = 4, int KG = 1, int STAG = 0, int DBG = 0>
__global__ __launch_bounds__(64 * NW * KG, 1) void gemm_rsf_kernel(RsArgs g) {
  using G = RsGeo<BM, BN, WGM, D, M32, NW>;
  constexpr int NTG = 64 * NW, NT = NTG * KG;       // threads per k-group / per workgroup
  static_assert(KG == 1 || KG == 2, "k-groups");
  static_assert(STAG == 0 || KG == 2, "stagger needs two k-groups");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave_all = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = KG == 1 ? 0 : wave_all / NW;      // wave-uniform
  const int wave = wave_all - grp * NW;
  const int tg = tid - grp * NTG;                   // thread index inside the k-group
  const int wm = wave % WGM, wn = wave / WGM;

  // ---- tile walk: XCD-major (workgroups b, b + 8, ... share an XCD under round-robin dispatch: speed
  // only), then groups of gm m-tiles x all n-tiles so an XCD's A and B panels share its L2
  const int tiles_n = g.N / BN, tiles_m = g.M / BM, tiles = tiles_m * tiles_n;
  const int L = blockIdx.x;
  const int idx = xcd_grouped(L, tiles);
  int mb, nb;
  if (g.gm > 1 && tiles_m % g.gm == 0) {
    const int span = g.gm * tiles_n, grp_ = idx / span, in = idx - grp_ * span;
    mb = grp_ * g.gm + in % g.gm;
    nb = in / g.gm;
  } else {
    mb = idx / tiles_n;
    nb = idx - mb * tiles_n;
  }
  const int m0 = mb * BM, n0 = nb * BN;
  const int nk = g.K / G::BK, nkg = nk / KG;        // k-steps in all / of this group
  DLTB_DCHECK(m0 + BM <= g.M && n0 + BN <= g.N && nk * G::BK == g.K && nkg % D == 0 && nkg >= 2);

  const int prow = tg >> 3, pch = tg & 7;
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
  const uint32_t ldsg = lds0 + grp * 3 * G::STAGE;  // this group's three stage buffers
  using E = RsEpiF<BM, BN, NT>;
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
  auto load1 = [&](int j, u32x4 (&r)[G::NI], int l) {
    // group-local k-step j -> global k-step j * KG + grp (past the end: the group's last stage again,
    // loaded into registers that are never written to a buffer anybody reads)
    const int so = (min(j, nkg - 1) * KG + grp) * (G::BK * 2);
    if (l < G::NA) r[l] = __builtin_amdgcn_raw_buffer_load_b128(ra, voa[l], so, 0);
    else r[l] = __builtin_amdgcn_raw_buffer_load_b128(rb, vob[l - G::NA], so, 0);
  };
  auto mma1 = [&](const Frags& F, int q) {
    const int s = q / (G::FM * G::FN), i = (q / G::FN) % G::FM, j = q % G::FN;
    if constexpr (M32) acc[i][j] = mfma32(F.f[s][G::FM + j], F.f[s][i], acc[i][j]);
    else acc[i][j] = mfma16(F.f[s][G::FM + j], F.f[s][i], acc[i][j]);
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
  for (int w = 0; w < G::NI; ++w) write1(ldsg, R[0], w);
#pragma unroll
  for (int l = 0; l < G::NI; ++l) load1(D, R[0], l);
#pragma unroll
  for (int w = 0; w < G::NI; ++w) write1(ldsg + G::STAGE, R[1 % D], w);
#pragma unroll
  for (int l = 0; l < G::NI; ++l) load1(D + 1, R[1 % D], l);
  rs_barrier();
#pragma unroll
  for (int r = 0; r < NR; ++r) read1(X, ldsg, 0, r);
  uint32_t b_cur = ldsg, b_nxt = ldsg + G::STAGE, b_wr = ldsg + 2 * G::STAGE;
  if constexpr (STAG) {
    if (grp == 1) __builtin_amdgcn_s_barrier();        // group 1 runs half a segment behind
  }

  for (int t = 0; t < nkg; t += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int j = t + u;
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
          if constexpr ((DBG & 16) == 0) load1(j + 2 + D, RR, w);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (STAG) {
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
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
  if constexpr (STAG) {
    if (grp == 0) __builtin_amdgcn_s_barrier();        // the barrier group 1 took before its loop
  }

  rs_barrier();                                          // all fragment reads done before the epilogue image
  static_assert(E::BYTES <= 3 * KG * G::STAGE, "epilogue image exceeds the stage buffers");
  auto put_all = [&](bool add) {
#pragma unroll
    for (int i = 0; i < G::FM; ++i) {
#pragma unroll
      for (int j = 0; j < G::FN; ++j) {
#pragma unroll
        for (int q = 0; q < G::ACC / 4; ++q) {
          const int ml = arow0 + G::T * i + fr, nl = brow0 + G::T * j + (M32 ? 8 * q + 4 * fq : 4 * fq);
          float a4[4] = {acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
          if (add) {
            const f32x4 o = E::get(lds0, ml, nl);
            a4[0] += o[0]; a4[1] += o[1]; a4[2] += o[2]; a4[3] += o[3];
          }
          E::put(lds0, ml, nl, a4);
        }
      }
    }
  };
  if constexpr (KG == 1) {
    put_all(false);
  } else {
    // group 1 parks its partial tile in the image, group 0 adds its own to it (the same lane -> element map)
    if (grp == 1) put_all(false);
    rs_barrier();
    if (grp == 0) put_all(true);
  }
  rs_barrier();
  E::flush(g, lds0, m0, n0, tid, pbias, paux);
}

template <int BM, int BN, int WGM, int D, bool M32, int NW = 4, int KG = 1, int STAG = 0, int DBG = 0>
void launch_rsf(const RsArgs& g, hipStream_t st) {
  constexpr int smem = 3 * KG * RsGeo<BM, BN, WGM, D, M32, NW>::STAGE;
  static_assert(smem <= 163840, "LDS budget");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_rsf_kernel<BM, BN, WGM, D, M32, NW, KG, STAG, DBG>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  const int tiles = (g.M / BM) * (g.N / BN);
  hipLaunchKernelGGL((gemm_rsf_kernel<BM, BN, WGM, D, M32, NW, KG, STAG, DBG>), dim3(tiles), dim3(64 * NW * KG),
                     smem, st, g);
}

struct RsCfg {
  int bm, bn, wgm, d;
  bool m32;
  int nw = 4;        // waves per k-group (8: the output tile split over 8 waves, 2 per SIMD)
  int kg = 1;        // k-groups (2: two 4-wave groups on the same tile, alternate k-steps)
  int stag = 0;      // k-groups staggered by half a segment
  int dbg = 0;       // != 0: timing-only ablation (wrong results by construction; refused unless DLTB_GEMM_ABLATION=1)
};
// The shipped table (configs/gemm_rs/gemm_rs_gfx950.csv) names configs by index.  Rounds 3-5 measured and
// retired the two-buffer, sched_group_barrier, direct-operand and loader/consumer variants (git history;
// profiles/gemm_rs_instep_ab_r5.txt, profiles/gemm_nt_r3.txt).
constexpr RsCfg kRsCfgs[] = {
    // 0-5: one 4-wave group.  0: 128 x 64, 32x32x16, 4 stages in flight (TinyGPT-A's N = 1024 products);
    // 1: 128 x 256; 2: 128 x 192 on 16x16x32; 3: 128 x 128; 4: 0 at 2 stages; 5: 0 with the waves 4 x 1
    {128, 64, 2, 4, true}, {128, 256, 2, 2, true}, {128, 192, 2, 2, false}, {128, 128, 2, 2, true},
    {128, 64, 2, 2, true}, {128, 64, 4, 4, true},
    // 6-8: 8 waves splitting the output tile (2 per SIMD): 128 x 256, 128 x 192 (16x16), 128 x 64 (4 x 2)
    {128, 256, 2, 2, true, 8}, {128, 192, 2, 2, false, 8}, {128, 64, 4, 4, true, 8},
    // 9-14: two 4-wave k-groups on one 128 x 64 tile: 32x32 at 2 / 4 stages per group, the same staggered,
    // 16x16x32 at 2 stages plain / staggered
    {128, 64, 2, 2, true, 4, 2, 0}, {128, 64, 2, 4, true, 4, 2, 0}, {128, 64, 2, 2, true, 4, 2, 1},
    {128, 64, 2, 4, true, 4, 2, 1}, {128, 64, 2, 2, false, 4, 2, 0}, {128, 64, 2, 2, false, 4, 2, 1},
    // 15-19: ablations of cfg 0 -- no fragment reads / no loop loads / no MFMA / no LDS writes / none of them
    {128, 64, 2, 4, true, 4, 1, 0, 8}, {128, 64, 2, 4, true, 4, 1, 0, 16}, {128, 64, 2, 4, true, 4, 1, 0, 32},
    {128, 64, 2, 4, true, 4, 1, 0, 64}, {128, 64, 2, 4, true, 4, 1, 0, 120},
    // 20-24: the same ablations of cfg 9
    {128, 64, 2, 2, true, 4, 2, 0, 8}, {128, 64, 2, 2, true, 4, 2, 0, 16}, {128, 64, 2, 2, true, 4, 2, 0, 32},
    {128, 64, 2, 2, true, 4, 2, 0, 64}, {128, 64, 2, 2, true, 4, 2, 0, 120},
};
constexpr int kRsNumCfgs = sizeof(kRsCfgs) / sizeof(kRsCfgs[0]);

void launch_rs_cfg(int cfg, const RsArgs& g, hipStream_t st) {
  switch (cfg) {
    case 0: launch_rsf<128, 64, 2, 4, true>(g, st); break;
    case 1: launch_rsf<128, 256, 2, 2, true>(g, st); break;
    case 2: launch_rsf<128, 192, 2, 2, false>(g, st); break;
    case 3: launch_rsf<128, 128, 2, 2, true>(g, st); break;
    case 4: launch_rsf<128, 64, 2, 2, true>(g, st); break;
    case 5: launch_rsf<128, 64, 4, 4, true>(g, st); break;
    case 6: launch_rsf<128, 256, 2, 2, true, 8>(g, st); break;
    case 7: launch_rsf<128, 192, 2, 2, false, 8>(g, st); break;
    case 8: launch_rsf<128, 64, 4, 4, true, 8>(g, st); break;
    case 9: launch_rsf<128, 64, 2, 2, true, 4, 2, 0>(g, st); break;
    case 10: launch_rsf<128, 64, 2, 4, true, 4, 2, 0>(g, st); break;
    case 11: launch_rsf<128, 64, 2, 2, true, 4, 2, 1>(g, st); break;
    case 12: launch_rsf<128, 64, 2, 4, true, 4, 2, 1>(g, st); break;
    case 13: launch_rsf<128, 64, 2, 2, false, 4, 2, 0>(g, st); break;
    case 14: launch_rsf<128, 64, 2, 2, false, 4, 2, 1>(g, st); break;
    case 15: launch_rsf<128, 64, 2, 4, true, 4, 1, 0, 8>(g, st); break;
    case 16: launch_rsf<128, 64, 2, 4, true, 4, 1, 0, 16>(g, st); break;
    case 17: launch_rsf<128, 64, 2, 4, true, 4, 1, 0, 32>(g, st); break;
    case 18: launch_rsf<128, 64, 2, 4, true, 4, 1, 0, 64>(g, st); break;
    case 19: launch_rsf<128, 64, 2, 4, true, 4, 1, 0, 120>(g, st); break;
    case 20: launch_rsf<128, 64, 2, 2, true, 4, 2, 0, 8>(g, st); break;
    case 21: launch_rsf<128, 64, 2, 2, true, 4, 2, 0, 16>(g, st); break;
    case 22: launch_rsf<128, 64, 2, 2, true, 4, 2, 0, 32>(g, st); break;
    case 23: launch_rsf<128, 64, 2, 2, true, 4, 2, 0, 64>(g, st); break;
    default: launch_rsf<128, 64, 2, 2, true, 4, 2, 0, 120>(g, st); break;
  }
}

}  // namespace

static bool rs_ablation_enabled() {
  static const bool on = [] {
    const char* e = getenv("DLTB_GEMM_ABLATION");
    return e && e[0] == '1';
  }();
  return on;
}

static bool rs_fits(int c, int M, int N, int K) {
  if (c < 0 || c >= kRsNumCfgs) return false;
  const RsCfg t = kRsCfgs[c];
  if (t.dbg != 0 && !rs_ablation_enabled()) return false;   // never a silent wrong product
  const int step = 64 * t.d * t.kg;
  return M > 0 && N > 0 && K > 0 && M % t.bm == 0 && N % t.bn == 0 && K % step == 0 && K / 64 >= 2 * t.kg;
}

int dltb_gemm_rs_pick(int M, int N, int K) {
  // the production config whose tile count is closest to one workgroup per CU (256); ties keep the earlier
  int best = -1, bestd = 1 << 30;
  for (int c = 0; c < kRsNumCfgs; ++c) {
    if (kRsCfgs[c].dbg != 0 || !rs_fits(c, M, N, K)) continue;
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
  // the aux / column-partial epilogue: a thread's columns fixed across rows, its aux values prefetched
  if (cfg < 0) cfg = dltb_gemm_rs_pick(M, N, K);
  if (!dltb_gemm_rs_supported(M, N, K, cfg)) return false;
  const int nt = 64 * kRsCfgs[cfg].nw * kRsCfgs[cfg].kg;
  const int cpr = kRsCfgs[cfg].bn / 4;
  return nt % cpr == 0 && kRsCfgs[cfg].bm * cpr / nt <= 16;   // RsEpiF::AUX_PF
}

bool dltb_gemm_rs_gelu_supported(int M, int N, int K, int cfg) {
  // the GELU-output epilogue: every config (fp32 epilogue image)
  if (cfg < 0) cfg = dltb_gemm_rs_pick(M, N, K);
  return dltb_gemm_rs_supported(M, N, K, cfg);
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
