// bf16 GEMM on MFMA for the transformer's linear layers (gfx950).
//
//   C[M, N] = sum_k A(m, k) B(k, n)   (+ bias[n])   (+ C  when accumulating)      fp32 accumulate
//
// Two operand layouts cover every product of a training step (see ops/functional.py):
//   NT: A stored [M][K], B stored [N][K]  (both K-contiguous)  forward x W^T, dgrad dY (W^T)^T
//   TN: A stored [K][M], B stored [K][N]  (both K-strided)     wgrad dY^T X
// so both operands of one kernel use the same fragment read (row_frag for NT, tr_frag for TN) and
// therefore the same k order inside an MFMA (mfma_tiles.h).
//
// Block = 4 waves (2 x 2), tile BM x BN x 64.  Per 64-deep k-step each wave does 4 k16 steps of
// (BM/64) x (BN/64) v_mfma_f32_32x32x16_bf16; A and B tiles are double-buffered in LDS and filled by
// LDS-DMA (global_load_lds_dwordx4, swizzle on the source address) one k-step ahead.  MFMA roles
// are swapped (srcA = B fragment, srcB = A fragment) so the accumulator has m on the lane and 4
// consecutive n per register group: the epilogue stores 8-byte bf16x4 vectors.
// The grid walks tiles XCD-major (consecutive workgroups go to different XCDs; each XCD gets a
// contiguous run of tiles sharing A rows in its L2).  Optional split-K writes fp32 partials
// reduced by a second kernel (small grids: out-proj / wgrad of 1024 x 1024).
#include "common.h"
#include "launchers.h"
#include "mfma_tiles.h"

namespace {

constexpr int kBK = 64;

struct GemmArgs {
  const bf16_t* a;
  const bf16_t* b;
  bf16_t* c;
  const bf16_t* bias;
  const float* alpha;   // optional device scalar multiplying A B (before bias / accumulate)
  float* part;          // split-K partials [splits][M][N] (fp32), null without split-K
  long lda, ldb, ldc;
  int M, N, K;
  int accumulate;
  int ksplit;           // K range per split (multiple of kBK)
  int pf;               // L2 prefetch distance in k-steps (PF kernels)
  int gm;               // tile order: groups of gm row-blocks (each XCD's run covers gm x (run / gm) tiles)
};

// tile image geometry: NT -> rows = m (or n), 64 k per row (D = 64 image, BM rows);
//                      TN -> rows = k (64), BM (or BN) m per row (D = BM image, 64 rows)
template <int BM, int BN, bool TN>
struct Geo {
  static constexpr int A_BYTES = BM * kBK * 2;
  static constexpr int B_BYTES = BN * kBK * 2;
  static constexpr int STAGE = A_BYTES + B_BYTES;
};

// NSTAGE >= 3: one workgroup per CU (a deep LDS-DMA ring, counted vmcnt across the barrier);
// NSTAGE == 2: a double buffer small enough for two workgroups per CU (one wave of each per SIMD:
// one wave's MFMAs cover the other's LDS reads and barrier waits).
template <int BM, int BN, bool TN, int NSTAGE, bool PF>
__global__ __launch_bounds__(256, NSTAGE == 2 ? 2 : 1) void gemm_kernel(GemmArgs g) {
  using G = Geo<BM, BN, TN>;
  constexpr int WM = BM / 2, WN = BN / 2;          // wave tile
  constexpr int FM = WM / 32, FN = WN / 32;        // 32x32 MFMA tiles per wave
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r = lane & 31;
  const int wm = w & 1, wn = w >> 1;
  const int wv = __builtin_amdgcn_readfirstlane(w);
  // ---- tile coordinates (XCD-major walk), split index
  const int tiles_n = g.N / BN, tiles = (g.M / BM) * tiles_n;
  const int splits = gridDim.x / tiles;
  int L = blockIdx.x;
  const int split = L / tiles;
  L -= split * tiles;
  int idx = L;
  if ((tiles & 7) == 0) idx = (L & 7) * (tiles >> 3) + (L >> 3);
  int mb = idx / tiles_n, nb = idx % tiles_n;
  const int tiles_m = g.M / BM;
  if (g.gm > 1 && tiles_m % g.gm == 0) {          // grouped order: gm row-blocks x all column-blocks
    const int grp = idx / (g.gm * tiles_n), in = idx % (g.gm * tiles_n);
    mb = grp * g.gm + in % g.gm;
    nb = in / g.gm;
  }
  const int m0 = mb * BM, n0 = nb * BN;
  const int kbeg = split * g.ksplit;
  const int nk = min(g.ksplit, g.K - kbeg) / kBK;
  DLTB_DCHECK(m0 + BM <= g.M && n0 + BN <= g.N && kbeg + nk * kBK <= g.K && nk > 0);

  // L2 prefetch of k-step kt + pf: one 4-byte LDS-DMA per 128-byte line of the stage (BM + BN lines),
  // landing in a scratch LDS slot.  The XCD's L2 then already holds the lines when the real stage is
  // issued, so the ring only has to cover L2 latency, not the Infinity-Cache latency of first touch.
  constexpr int NPF = PF ? (BM + BN + 255) / 256 : 0;
  auto prefetch = [&](int kt) {
    const int kp = kbeg + min(kt + g.pf, nk - 1) * kBK;
#pragma unroll
    for (int i = 0; i < NPF; ++i) {
      int t = (i * 256 + tid) % (BM + BN);
      const bf16_t* src;
      if constexpr (!TN) {
        src = t < BM ? g.a + (long)(m0 + t) * g.lda + kp : g.b + (long)(n0 + t - BM) * g.ldb + kp;
      } else {
        if (t < BM) src = g.a + (long)(kp + t / (BM / 64)) * g.lda + m0 + (t % (BM / 64)) * 64;
        else { t -= BM; src = g.b + (long)(kp + t / (BN / 64)) * g.ldb + n0 + (t % (BN / 64)) * 64; }
      }
      glds4_asm(src, smem + NSTAGE * G::STAGE + wv * 256);
    }
  };

  auto load_stage = [&](int kt, int st) {
    if constexpr (PF) prefetch(kt);
    char* sa = smem + st * G::STAGE;
    char* sb = sa + G::A_BYTES;
    const int k0 = kbeg + kt * kBK;
    if constexpr (!TN) {
      GldsTile<64, BM, true>::load(g.a + k0, g.lda, m0, sa, wv, lane);
      GldsTile<64, BN, true>::load(g.b + k0, g.ldb, n0, sb, wv, lane);
    } else {
      GldsTile<BM, kBK, true>::load(g.a + m0, g.lda, k0, sa, wv, lane);
      GldsTile<BN, kBK, true>::load(g.b + n0, g.ldb, k0, sb, wv, lane);
    }
  };

  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x16{};

  // NSTAGE-deep LDS ring filled by LDS-DMA.  Each wave issues GLDS wave-instructions per stage;
  // a COUNTED vmcnt (not __syncthreads' vmcnt(0)) retires only the stage about to be read, so the
  // next NSTAGE-2 stages stay in flight across the raw s_barrier.
  constexpr int GLDS = NPF + (TN ? (GldsTile<BM, kBK>::NI + GldsTile<BN, kBK>::NI)
                                : (GldsTile<64, BM>::NI + GldsTile<64, BN>::NI));
#pragma unroll
  for (int st = 0; st < NSTAGE - 1; ++st)
    if (st < nk) load_stage(st, st);
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = min(nk - 1 - kt, NSTAGE - 2);     // stages issued after kt that may stay in flight
    if (ahead >= 2) wait_vm<2 * GLDS>();
    else if (ahead == 1) wait_vm<GLDS>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();                       // every wave's part of stage kt has landed
    if (kt + NSTAGE - 1 < nk) load_stage(kt + NSTAGE - 1, (kt + NSTAGE - 1) % NSTAGE);
    const char* sa = smem + (kt % NSTAGE) * G::STAGE;
    const char* sb = sa + G::A_BYTES;
#pragma unroll
    for (int s = 0; s < kBK / 16; ++s) {
      bfx8 fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        if constexpr (!TN) fa[i] = row_frag<64>(sa, wm * WM + 32 * i + r, 2 * s + h);
        else fa[i] = tr_frag<BM>(sa, 16 * s, wm * WM + 32 * i, lane);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        if constexpr (!TN) fb[j] = row_frag<64>(sb, wn * WN + 32 * j + r, 2 * s + h);
        else fb[j] = tr_frag<BN>(sb, 16 * s, wn * WN + 32 * j, lane);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma32(fb[j], fa[i], acc[i][j]);   // lane <-> m
    }
    // the NEXT iteration's barrier orders these LDS reads before stage kt's buffer is refilled
  }

  // ---- epilogue: lane -> row m, register group q -> columns n .. n+3
  const float al = (g.alpha && splits == 1) ? *g.alpha : 1.f;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = m0 + wm * WM + 32 * i + r;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = n0 + wn * WN + 32 * j + 8 * q + 4 * h;
        float v[4] = {acc[i][j][4 * q] * al, acc[i][j][4 * q + 1] * al, acc[i][j][4 * q + 2] * al,
                      acc[i][j][4 * q + 3] * al};
        if (splits > 1) {
          *reinterpret_cast<float4*>(g.part + ((size_t)split * g.M + m) * g.N + n) = make_float4(v[0], v[1], v[2], v[3]);
          continue;
        }
        if (g.bias) {
          const uint2 bb = *reinterpret_cast<const uint2*>(g.bias + n);
          v[0] += lo_bf(bb.x); v[1] += hi_bf(bb.x); v[2] += lo_bf(bb.y); v[3] += hi_bf(bb.y);
        }
        bf16_t* cp = g.c + (size_t)m * g.ldc + n;
        if (g.accumulate) {
          const uint2 old = *reinterpret_cast<const uint2*>(cp);
          v[0] += lo_bf(old.x); v[1] += hi_bf(old.x); v[2] += lo_bf(old.y); v[3] += hi_bf(old.y);
        }
        uint2 o;
        o.x = pack_bf2(v[0], v[1]);
        o.y = pack_bf2(v[2], v[3]);
        *reinterpret_cast<uint2*>(cp) = o;
      }
    }
  }
}

// split-K reduction: C = sum_s part[s] (+ bias) (+ C)
__global__ __launch_bounds__(256) void gemm_splitk_reduce(GemmArgs g, int splits) {
  const long total4 = (long)g.M * g.N / 4;
  const float al = g.alpha ? *g.alpha : 1.f;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total4; i += (long)gridDim.x * 256) {
    const long e = i * 4;
    const int m = (int)(e / g.N), n = (int)(e % g.N);
    float4 s = *reinterpret_cast<const float4*>(g.part + e);
    for (int k = 1; k < splits; ++k) {
      const float4 t = *reinterpret_cast<const float4*>(g.part + (size_t)k * g.M * g.N + e);
      s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
    }
    float v[4] = {s.x * al, s.y * al, s.z * al, s.w * al};
    if (g.bias) {
      const uint2 bb = *reinterpret_cast<const uint2*>(g.bias + n);
      v[0] += lo_bf(bb.x); v[1] += hi_bf(bb.x); v[2] += lo_bf(bb.y); v[3] += hi_bf(bb.y);
    }
    bf16_t* cp = g.c + (size_t)m * g.ldc + n;
    if (g.accumulate) {
      const uint2 old = *reinterpret_cast<const uint2*>(cp);
      v[0] += lo_bf(old.x); v[1] += hi_bf(old.x); v[2] += lo_bf(old.y); v[3] += hi_bf(old.y);
    }
    uint2 o;
    o.x = pack_bf2(v[0], v[1]);
    o.y = pack_bf2(v[2], v[3]);
    *reinterpret_cast<uint2*>(cp) = o;
  }
}

template <int BM, int BN, bool TN, bool PF, int NSTAGE>
void launch_ns(const GemmArgs& g, int splits, hipStream_t st) {
  constexpr int smem = NSTAGE * Geo<BM, BN, TN>::STAGE + (PF ? 1024 : 0);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_kernel<BM, BN, TN, NSTAGE, PF>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  const int tiles = (g.M / BM) * (g.N / BN);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, TN, NSTAGE, PF>), dim3(tiles * splits), dim3(256), smem, st, g);
}

// stages == 2: double buffer (two or more workgroups per CU); otherwise the deep ring (<= 128 KiB,
// one workgroup per CU)
template <int BM, int BN, bool TN, bool PF>
void launch_pf(const GemmArgs& g, int splits, int stages, hipStream_t st) {
  constexpr int DEEP = Geo<BM, BN, TN>::STAGE <= 32768 ? 4 : 3;
  if (stages == 2) launch_ns<BM, BN, TN, PF, 2>(g, splits, st);
  else launch_ns<BM, BN, TN, PF, DEEP>(g, splits, st);
}

template <int BM, int BN, bool TN>
void launch_t(const GemmArgs& g, int splits, int stages, hipStream_t st) {
  if (g.pf > 0) launch_pf<BM, BN, TN, true>(g, splits, stages, st);
  else launch_pf<BM, BN, TN, false>(g, splits, stages, st);
}

}  // namespace

// tile configs (BM x BN): 0 = 128x128, 1 = 256x128, 2 = 128x256, 3 = 128x64, 4 = 64x128, 5 = 64x64
static void cfg_tile(int cfg, int& BM, int& BN) {
  static const int t[6][2] = {{128, 128}, {256, 128}, {128, 256}, {128, 64}, {64, 128}, {64, 64}};
  if (cfg < 0 || cfg > 5) cfg = 0;
  BM = t[cfg][0];
  BN = t[cfg][1];
}

bool dltb_gemm_supported(int M, int N, int K, bool tn, int cfg) {
  if (cfg < 0 || cfg > 5) return false;
  int BM, BN;
  cfg_tile(cfg, BM, BN);
  if (tn && (BM > 128 || BN > 128)) return false;   // TN images are <= 128-element rows (mfma_tiles.h swizzle)
  return M % BM == 0 && N % BN == 0 && K % kBK == 0 && M > 0 && N > 0 && K > 0;
}

int dltb_gemm(const void* a, const void* b, void* c, const void* bias, float* part, long lda, long ldb,
              long ldc, int M, int N, int K, bool tn, int accumulate, int splits, int cfg, int pf, int gm,
              const float* alpha, hipStream_t st, int stages) {
  GemmArgs g{};
  g.alpha = alpha;
  g.pf = pf;
  g.gm = gm;
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
  g.accumulate = accumulate;
  if (splits < 1) splits = 1;
  const int kchunks = K / kBK;
  if (splits > kchunks) splits = kchunks;
  g.ksplit = ((kchunks + splits - 1) / splits) * kBK;
  splits = (K + g.ksplit - 1) / g.ksplit;
  g.part = splits > 1 ? part : nullptr;
  if (splits > 1 && !part) return -1;
#define DLTB_G(BM, BN)                                              \
  do {                                                              \
    if (tn) launch_t<BM, BN, true>(g, splits, stages, st);          \
    else launch_t<BM, BN, false>(g, splits, stages, st);            \
  } while (0)
  switch (cfg) {
    case 1: launch_t<256, 128, false>(g, splits, stages, st); break;
    case 2: launch_t<128, 256, false>(g, splits, stages, st); break;
    case 3: DLTB_G(128, 64); break;
    case 4: DLTB_G(64, 128); break;
    case 5: DLTB_G(64, 64); break;
    default: DLTB_G(128, 128); break;
  }
#undef DLTB_G
  if (splits > 1) {
    long total4 = (long)M * N / 4;
    long grid = (total4 + 255) / 256;
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL(gemm_splitk_reduce, dim3(grid), dim3(256), 0, st, g, splits);
  }
  return splits;
}
