// bf16 "TN" GEMM for weight gradients (gfx950, CDNA4):
//
//   C[b][M][N] (+)= sum_k A[b][k][m] . B[b][k][n]          fp32 accumulate, bf16 out
//
// A weight gradient dW = dY^T X has the token (reduction) index as the OUTER dimension of both operands
// (dY [T][out], X [T][in], both row-major), so neither operand is K-contiguous.  hipBLASLt runs that layout
// 25-45 % slower than the K-contiguous one (profiles/gemm_layouts_r2.txt: 1.03-1.04 against 1.48-1.52
// PFLOP/s on the same shapes; the TinyGPT-A window-wide batched dW at 1.07-1.17).  Here the operands
// are staged as they lie -- 32 token rows x 256 feature columns per operand and k-step, filled by LDS-DMA
// (global_load_lds_dwordx4, 1 KiB = two 512-byte rows per wave-instruction) -- and the MFMA fragments
// are read TRANSPOSED out of LDS with ds_read_b64_tr_b16, which hands each lane 4 consecutive tokens of
// one feature column: the layout costs no extra pass and no extra LDS traffic.
//
// Tile 256 (m) x 256 (n), 512 threads = 8 waves as 2 (m) x 4 (n), each wave 128 x 64 outputs on
// v_mfma_f32_16x16x32_bf16 (8 x 4 accumulators).  MFMA operands swapped (the X fragment is the MFMA's A
// operand), so a lane holds 4 consecutive n of one m: 8-byte epilogue stores.  The DMA of a stage runs two
// to three k-steps ahead (counted vmcnt, raw s_barrier: the loads stay in flight across the barrier).
//
// LDS image of one operand and stage: [32 k][256 cols] bf16, 512-byte rows; the 32-byte segment s (16
// columns) of row k is stored at segment s ^ h(k), h(k) = (k & 3) | ((k >> 3) & 1) << 2.  A transposed
// read of one 32-lane half touches 8 rows (k = 8g + q + 4hh over g = 0, 1 and q = 0..3) of one column
// segment: h maps them to the 8 distinct 32-byte bank segments of a 256-byte bank row (conflict-free).
// The swizzle is applied on the DMA's SOURCE address (the LDS side of an LDS-DMA is lane-linear).
#include "common.h"
#include "launchers.h"
#include "mfma_tiles.h"

namespace {

constexpr int kTM = 256, kTN = 256;
constexpr int kRowB = 512;                    // bytes per k-row of an operand image (256 bf16)

struct TnArgs {
  const bf16_t* a;
  const bf16_t* b;
  bf16_t* c;
  long lda, ldb, ldc;                         // row strides (elements)
  long sa, sb, sc;                            // batch strides (elements)
  int M, N, K, batch;
  int accumulate;
};

typedef __attribute__((ext_vector_type(4))) float f4;

DLTB_DEV f4 mfma16(bfx8 a, bfx8 b, f4 c) {
#if DLTB_F16
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
#else
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
#endif
}

DLTB_DEV int tn_h(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }

// workgroup barrier that is also a compiler barrier for LDS accesses (no read of a stage may be moved
// across the barrier that orders it against the DMA refilling that stage)
DLTB_DEV void tn_barrier() { asm volatile("s_barrier" ::: "memory"); }

// one operand fragment (16 columns x 32 k) by two transposed reads at lane byte offset `off` of a stage
// image: element j of lane l = image[k0 + 8 (l >> 4) + j][column c0 + (l & 15)]
template <int OFF>
DLTB_DEV bfx8 tn_frag(uint32_t base, uint32_t off) {
  return tr_frag_at<OFF>(base + off, base + off + 4 * kRowB);
}

// The main loop: 32-deep k-steps in a ring of four 32 KiB stages (128 KiB), two fragment register sets.  Step kt
// computes stage kt from registers (read during step kt - 1) while reading stage kt + 1's fragments into
// the other set, and refills the buffer stage kt's fragments came from with stage kt + 4 (every wave read
// it before the barrier that ended step kt - 1); one barrier per step publishes stage kt + 2 (its DMA was
// issued two steps earlier; stages kt + 3 / kt + 4 stay in flight across it).  No fragment read is exposed
// at a step boundary.  (Measured against it on the dW shapes, profiles/gemm_tn_r6.txt: 64-deep k-steps in
// two stage buffers with two barriers per step, 8-10 % slower; the same with one barrier and the second
// substep's reads pipelined, 3-5 % slower; the refill's DMA spread over the MFMA groups and s_setprio
// around them, within +-2 %; the loop made branch-free, -1.5 %; four waves of 128 x 128 outputs (one wave per
// SIMD, 64 MFMAs against 16 fragment reads per k-step, the 256 accumulators pinned in AGPRs by inline-asm
// MFMAs), 2 % slower; v_mfma_f32_32x32x16 (16 instead of 32 MFMAs per wave and k-step for the same reads, twice
// the issue cycles between them; 64-byte-segment swizzle), 2 % slower.  The MFMA stream alone, with this kernel's 8 x 4 distinct fragments and 32 accumulators
// per wave, sustains 2.04 PF/s on random data (scripts/probes/mfma_peak_probe.hip).)
constexpr int kTK3 = 32;
constexpr int kImg3 = kTK3 * kRowB;           // 16 KiB
constexpr int kStage3 = 2 * kImg3;            // 32 KiB
constexpr int kRing3 = 4;
constexpr int kGlds3 = kImg3 / 1024 / 8;      // 2 per wave, operand and stage

__global__ __launch_bounds__(512, 1) void gemm_tn_kernel(TnArgs g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int tm = g.M / kTM, tn = g.N / kTN, per = tm * tn, tiles = per * g.batch;
  const int L = blockIdx.x;
  const int idx = xcd_grouped(L, tiles);
  const int bt = idx / per, rem = idx - bt * per;
  const int mb = rem / tn, nb = rem - mb * tn;
  const int m0 = mb * kTM, n0 = nb * kTN;
  const int nk = g.K / kTK3;
  DLTB_DCHECK(bt < g.batch && m0 + kTM <= g.M && n0 + kTN <= g.N && nk * kTK3 == g.K && nk >= 4 && nk % 2 == 0);

  const bf16_t* abase = g.a + (long)bt * g.sa + m0;
  const bf16_t* bbase = g.b + (long)bt * g.sb + n0;
  uint32_t oa[kGlds3], ob[kGlds3];
#pragma unroll
  for (int i = 0; i < kGlds3; ++i) {
    const int row = 2 * (wave * kGlds3 + i) + (lane >> 5), c = lane & 31;
    const int col = (((c >> 1) ^ tn_h(row)) << 4) + (c & 1) * 8;
    oa[i] = (uint32_t)((row * g.lda + col) * 2);
    ob[i] = (uint32_t)((row * g.ldb + col) * 2);
  }
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) char*)smem;
  // stage kt into ring slot kt & 3: the wave's 2 + 2 LDS-DMA pieces from ONE asm block (m0 saved once, the four
  // destinations as immediates off the slot base), the sources as running wave-uniform pointers advanced one stage
  // per issue and clamped at the last stage (a refill nobody reads: the loop needs no branch and one uniform vmcnt
  // wait per step).  The per-piece form spent ~55 scalar instructions per step on 64-bit address products,
  // generic -> LDS pointer conversions and m0 save / restore.
  static_assert(kGlds3 == 2 && kImg3 == 0x4000, "issue() hard-codes two 1 KiB pieces per operand");
  const uint64_t astride = (uint64_t)kTK3 * g.lda * 2, bstride = (uint64_t)kTK3 * g.ldb * 2;
  uint64_t pa = uniform_ptr(abase), pb = uniform_ptr(bbase);   // stage to issue next
  const uint32_t ldsw = lds0 + (uint32_t)(wave * kGlds3 * 1024);
  auto issue = [&](int kt) {
    const uint32_t lds = ldsw + (uint32_t)((kt & (kRing3 - 1)) * kStage3);
    // destinations computed outside the asm: an s_add inside it would clobber SCC under a live compare
    const uint32_t l1 = lds + 0x400, l2 = lds + 0x4000, l3 = lds + 0x4400;
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %[keep], m0\n\t"
        "s_mov_b32 m0, %[l0]\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %[va0], %[sa]\n\t"
        "s_mov_b32 m0, %[l1]\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %[va1], %[sa]\n\t"
        "s_mov_b32 m0, %[l2]\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %[vb0], %[sb]\n\t"
        "s_mov_b32 m0, %[l3]\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %[vb1], %[sb]\n\t"
        "s_mov_b32 m0, %[keep]"
        : [keep] "=&s"(keep)
        : [va0] "v"(oa[0]), [va1] "v"(oa[1]), [vb0] "v"(ob[0]), [vb1] "v"(ob[1]), [sa] "s"(pa), [sb] "s"(pb),
          [l0] "s"(lds), [l1] "s"(l1), [l2] "s"(l2), [l3] "s"(l3)
        : "memory");
    const bool more = kt + 1 < nk;                // advance unless this was the last real stage
    pa += more ? astride : 0;
    pb += more ? bstride : 0;
  };
  const int fg = lane >> 4, fq = (lane >> 2) & 3, fp = lane & 3;
  const int hq = fq | ((fg & 1) << 2);
  const uint32_t rowoff = (uint32_t)((8 * fg + fq) * kRowB + 8 * fp);
  uint32_t offm[8], offn[4];
#pragma unroll
  for (int i = 0; i < 8; ++i) offm[i] = rowoff + ((((wm * 128 + 16 * i) >> 4) ^ hq) << 5);
#pragma unroll
  for (int j = 0; j < 4; ++j) offn[j] = kImg3 + rowoff + ((((wn * 64 + 16 * j) >> 4) ^ hq) << 5);

  f4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  auto read_all = [&](int kt, bfx8 (&fa)[8], bfx8 (&fb)[4]) {
    const uint32_t base = lds0 + (kt & (kRing3 - 1)) * kStage3;
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = tn_frag<0>(base, offn[j]);
#pragma unroll
    for (int i = 0; i < 8; ++i) fa[i] = tn_frag<0>(base, offm[i]);
  };
  // one step: MFMAs of stage kt (ca / cb) || fragments of stage kt + 1 (na / nb); refill; publish kt + 2.
  // Branch-free: the last step's reads of "stage nk" land in registers nobody uses, and the clamped refills
  // keep the in-flight count uniform (stages kt + 3 and kt + 4 may stay in flight across the barrier).
  auto step = [&](int kt, bfx8 (&ca)[8], bfx8 (&cb)[4], bfx8 (&na)[8], bfx8 (&nb)[4]) {
    issue(kt + 4);                                // into stage kt's buffer (read during step kt - 1)
    const uint32_t nbase = lds0 + ((kt + 1) & (kRing3 - 1)) * kStage3;
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(cb[j], ca[i], acc[i][j]);
      __builtin_amdgcn_sched_barrier(0);
      if (i < 4) nb[i] = tn_frag<0>(nbase, offn[i]);
      na[i] = tn_frag<0>(nbase, offm[i]);
      __builtin_amdgcn_sched_barrier(0);
    }
    wait_vm<4 * kGlds3>();                        // stage kt + 2 landed for this wave
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    tn_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  // prologue: stages 0..3 in flight; 0 and 1 published; stage 0's fragments in set A
#pragma unroll
  for (int s = 0; s < kRing3; ++s) issue(s);
  wait_vm<4 * kGlds3>();                       // stages 0, 1 landed (2, 3 in flight)
  tn_barrier();
  bfx8 fa0[8], fb0[4], fa1[8], fb1[4];
  read_all(0, fa0, fb0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  tn_barrier();                                // every wave read stage 0: step 0 may refill its buffer
  __builtin_amdgcn_sched_barrier(0);
  for (int kt = 0; kt < nk; kt += 2) {
    step(kt, fa0, fb0, fa1, fb1);
    step(kt + 1, fa1, fb1, fa0, fb0);
  }
  wait_vm<0>();

  const int er = lane & 15, eg = lane >> 4;
  bf16_t* cbase = g.c + (long)bt * g.sc + (long)(m0 + wm * 128 + er) * g.ldc + n0 + wn * 64 + 4 * eg;
  auto store = [&](int i, int j, const float (&v)[4]) {
    uint2 o;
    o.x = pack_bf2(v[0], v[1]);
    o.y = pack_bf2(v[2], v[3]);
    *reinterpret_cast<uint2*>(cbase + (long)(16 * i) * g.ldc + 16 * j) = o;
  };
  if (g.accumulate) {
    // every old value in flight at once (the fragment registers are dead here): one memory latency per tile
    // instead of one per fragment (a load -> wait -> store chain cost the head's wgrad ~20 us in the step)
    uint2 old[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) old[i][j] = *reinterpret_cast<const uint2*>(cbase + (long)(16 * i) * g.ldc + 16 * j);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float v[4] = {acc[i][j][0] + lo_bf(old[i][j].x), acc[i][j][1] + hi_bf(old[i][j].x),
                            acc[i][j][2] + lo_bf(old[i][j].y), acc[i][j][3] + hi_bf(old[i][j].y)};
        store(i, j, v);
      }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        store(i, j, v);
      }
  }
}

}  // namespace

bool dltb_gemm_tn_supported(int M, int N, int K) {
  return M > 0 && N > 0 && K > 0 && M % kTM == 0 && N % kTN == 0 && K % (2 * kTK3) == 0 && K / kTK3 >= 4;
}

int dltb_gemm_tn(const void* a, const void* b, void* c, long lda, long ldb, long ldc, long sa, long sb, long sc,
                 int M, int N, int K, int batch, int accumulate, hipStream_t st) {
  if (!dltb_gemm_tn_supported(M, N, K) || batch < 1) return -1;
  TnArgs g{};
  g.a = (const bf16_t*)a;
  g.b = (const bf16_t*)b;
  g.c = (bf16_t*)c;
  g.lda = lda;
  g.ldb = ldb;
  g.ldc = ldc;
  g.sa = sa;
  g.sb = sb;
  g.sc = sc;
  g.M = M;
  g.N = N;
  g.K = K;
  g.batch = batch;
  g.accumulate = accumulate;
  constexpr int smem = kRing3 * kStage3;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_tn_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  const dim3 grid((unsigned)((long)(M / kTM) * (N / kTN) * batch));
  hipLaunchKernelGGL(gemm_tn_kernel, grid, dim3(512), smem, st, g);
  return 0;
}
