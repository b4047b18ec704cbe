// Flash attention forward + backward for gfx950 (CDNA4), bf16 in / fp32 accumulate.
//
// Replaces the reference's nn.MultiheadAttention core (train_harness.py:114-116,127; torch
// functional.py:6576-6606): softmax(Q K^T / sqrt(D)) with dropout p on the probabilities, NON-causal
// for TinyGPT (the reference passes no mask) and causal + GQA for the Mistral shape.  The T x T
// probability matrix is never materialised (O(T) memory) and the head-averaged weights the
// reference computes and discards are not computed at all.
//
// Layout: q/k/v/o are token-major rows ([B*T, row_stride]) with head h at column h*D, so the
// kernels read the fused in_proj output [B*T, 3*d] directly and write dQ/dK/dV straight into the
// fused dqkv gradient.  lse: [B, Hq, T] (natural log), delta: [B, Hq, T].
//
// MFMA: v_mfma_f32_32x32x16_bf16 throughout, 4 waves / workgroup, 32 rows per wave.
//   forward  : S^T = K Q^T   (key on the MFMA row, query on the lane -> per-lane softmax, one
//              lane^32 exchange per row), O^T += V^T P^T with the P accumulator used directly
//              as the B operand (no LDS round trip) and V^T read by ds_read_b64_tr_b16.
//   dK/dV    : key-major; S = Q K^T, dP = dO V^T with K, V in registers; dV^T += dO^T Pdrop,
//              dK^T += Q^T dS, Q^T / dO^T by transposed LDS reads; GQA groups summed in-register.
//   dQ       : query-major; S^T, dP^T as in the forward, dQ^T += K^T dS^T.  No float atomics.
// LDS tiles are 64 rows x D bf16, dense, with a 16-byte-chunk XOR swizzle chosen so both the
// ds_read_b128 row-fragment reads and the ds_read_b64_tr_b16 transposed reads are bank-conflict
// free (D=64: chunk ^ (((r>>1)&1)<<2 | (r>>2)&3); D=128: chunk ^ ((r&3)<<2 | (r>>2)&3)).
// K/V (or Q/dO) tiles are double-buffered: global loads for tile t+1 are issued into registers
// before the MFMA work on tile t and written to LDS after it.
// Dropout uses the attention-site counter hash of common.h (rng_attn_pair; row = (b*Hq + h)*T + q, col = key).  The keep-mask is
// generated ONCE per call by a full-occupancy kernel as packed bits laid out for the forward's lane
// mapping: word (bh, t, h, q) holds, in bit 16n + i, the decision for key 64t + 32n + (i&3) +
// 8(i>>2) + 4h of query q — so forward and dQ lanes read one coalesced word per 64-key tile and the
// dK/dV kernel stages 4 words per query row in LDS.  The hash runs 1x instead of 3x, and the
// softmax kernels pay for dropout 1.5 VALU ops per probability in the forward (on the packed bf16
// P pairs, attn_mask.h) and 2 in the backward.  The softmax scale c = scale * log2(e) is folded into
// the operand each wave holds in registers (Q in the forward and dQ, K in dK/dV) and the row
// constants (-m, -lse log2 e, -delta/s) are the S / dP chains' initial accumulators, so the score
// tiles come out of the MFMAs as exp2 arguments.
#include <cstdlib>

// Softmax math is scalar f32: the file is built with -fno-slp-vectorize so the compiler does not
// pack it into v_pk_* ops, which beside MFMAs cost more issue time than the two scalar ops they
// replace (docs/MI355X_HW_NOTES.md, packed f32 VALU beside MFMAs; measured 1-3 % slower,
// profiles/attention_ab_r2.txt).
// The dK/dV kernel at D = 128 computes S / dP of both 32-row sub-tiles of a 64-row tile before the
// first softmax, so one sub-tile's MFMAs run under the other's VALU softmax; at D = 64 sub-tile after
// sub-tile measured equal or faster (TinyGPT-A dK/dV 56.2-57.2 vs 58.5-59.0 us, profiles/attention_ab_r2.txt;
// the D = 64 both-sub-tile variants of dK/dV and dQ were removed in round 6).
#ifndef DLTB_ATTN_LPT
#define DLTB_ATTN_LPT 1   // causal fwd / dQ grids heaviest-first (profiles/attn_lpt_order_m7b_r3.txt)
#endif
// key splits per workgroup at D = 64 (A/B builds: csrc/build.py --tag T -D DLTB_FWD_KS64=3); 4: 16 waves at
// 128 VGPRs without scratch, 1.5 % faster than 3 (profiles/splitk_planes_inline_ab_r4.txt)
#ifndef DLTB_FWD_KS64
#define DLTB_FWD_KS64 4
#endif
// causal D = 64 caps the splits at 3 (forward) / 2 (dQ) -- A/B build: -D DLTB_CAUSAL_KS_CAP=0
#ifndef DLTB_CAUSAL_KS_CAP
#define DLTB_CAUSAL_KS_CAP 1
#endif
#ifndef DLTB_DQ_KS64
#define DLTB_DQ_KS64 3
#endif
#include "attn_mask.h"
#include "common.h"
#include "mfma_tiles.h"

namespace {

constexpr float kLog2e = 1.4426950408889634f;
constexpr int kBlockRows = 128;   // query (fwd, dq) or key (dkdv) rows per workgroup
constexpr int kTile = 64;         // rows per streamed LDS tile

struct AttnArgs {
  const bf16_t* q;
  const bf16_t* k;
  const bf16_t* v;
  const bf16_t* o;
  const bf16_t* dout;
  bf16_t* out;      // fwd: O ; bwd_dq: dQ ; bwd_dkdv: dK
  bf16_t* out2;     // bwd_dkdv: dV
  float* lse;
  const float* delta;
  const uint32_t* mask;   // packed dropout keep-bits (see header), null without dropout
  long q_stride, k_stride, v_stride, o_stride, do_stride, out_stride, out2_stride;
  int B, T, Hq, Hkv;
  float scale;
  int causal;
  uint32_t thr16;
  float drop_scale;
  const int64_t* seed_ptr;
  int64_t site;
  int gsplit;       // bwd_dkdv: workgroups per KV head, each summing G / gsplit query heads
  float* part;      // bwd_dkdv with gsplit > 1: fp32 partials [gsplit][2][B*T][Hkv*D] (scaled)
};

// accumulator registers 8s .. 8s+7 -> bf16 B operand of k-step s
DLTB_DEV bfx8 acc_to_frag(const f32x16& x, int s) {
  bfx8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (h16_t)x[8 * s + j];
  return f;
}

// cooperative 64-row tile loader: 256 threads, 16-byte chunks
template <int D>
struct TileLoader {
  static constexpr int CH = D / 8;                    // chunks per row
  static constexpr int N = kTile * CH / 256;          // chunks per thread
  uint4 r[N];
  DLTB_DEV void load(const bf16_t* base, long stride, int row0, int tid) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int cid = tid + i * 256;
      const int row = cid / CH, ch = cid % CH;
      r[i] = ld16<uint4>(base + (long)(row0 + row) * stride + ch * 8);
    }
  }
  DLTB_DEV void store(char* tile, int tid) const {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int cid = tid + i * 256;
      const int row = cid / CH, ch = cid % CH;
      *reinterpret_cast<uint4*>(tile + toff<D>(row, ch)) = r[i];
    }
  }
};

// store a transposed 32x32-per-dt accumulator set: lane (row = lane & 31, h), reg i ->
// column dt*32 + (i&3) + 8(i>>2) + 4h, scaled
template <int D>
DLTB_DEV void store_acc_rows(bf16_t* dst_row, const f32x16* acc, float scale, int h) {
  // lanes r and r + 32 hold the two 4-column halves of each 8-column chunk of row r: one v_permlane32_swap per
  // dword hands lane r the chunk of group g0 and lane r + 32 that of g0 + 1, so every lane stores 16 bytes
  // (D / 16 dwordx4 stores instead of D / 8 dwordx2: the epilogue store tail is issue-bound).  All 64 lanes
  // must be active (every caller stores from wave-uniform control flow).
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt) {
#pragma unroll
    for (int g0 = 0; g0 < 4; g0 += 2) {
      const uint32_t x0 = pack_bf2(acc[dt][4 * g0 + 0] * scale, acc[dt][4 * g0 + 1] * scale);
      const uint32_t x1 = pack_bf2(acc[dt][4 * g0 + 2] * scale, acc[dt][4 * g0 + 3] * scale);
      const uint32_t y0 = pack_bf2(acc[dt][4 * g0 + 4] * scale, acc[dt][4 * g0 + 5] * scale);
      const uint32_t y1 = pack_bf2(acc[dt][4 * g0 + 6] * scale, acc[dt][4 * g0 + 7] * scale);
      const auto s0 = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
      const auto s1 = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
      const uint4 o = {s0[0], s1[0], s0[1], s1[1]};
      *reinterpret_cast<uint4*>(dst_row + dt * 32 + 8 * (g0 + h)) = o;
    }
  }
}

template <int D>
DLTB_DEV void store_acc_rows_f32(float* dst_row, const f32x16* acc, float scale, int h) {
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 o = {acc[dt][4 * g + 0] * scale, acc[dt][4 * g + 1] * scale,
                        acc[dt][4 * g + 2] * scale, acc[dt][4 * g + 3] * scale};
      *reinterpret_cast<float4*>(dst_row + dt * 32 + 8 * g + 4 * h) = o;
    }
  }
}

// =============================================================================== dropout mask
// (layout and body: attn_mask.h)
static_assert(kTile == kMaskKeyTile, "the packed mask tiles keys like the attention kernels");
__global__ __launch_bounds__(256) void attn_mask_kernel(uint32_t* __restrict__ mask, int T, uint32_t thr16,
                                                        const int64_t* __restrict__ seed_ptr, int64_t site) {
  // grid: x = query chunks of 256, y = (bh * nT + t) * 2 + h  (32-bit index math only)
  attn_mask_word(mask, T, thr16, seed_ptr, site, blockIdx.x * 256 + threadIdx.x, blockIdx.y);
}

// =============================================================================== forward
// Workgroup = KS key-splits x 4 waves; wave (qw, sp) owns query rows q0 .. q0+31 and the key tiles
// t == sp (mod KS).  KS = 2 doubles the waves per query block (2 waves / SIMD even at B*Hq*T/128
// = 256 workgroups, TinyGPT-A's shape); the two partial (m, l, O) states merge through LDS.
// Online softmax with a lazy rescale: the running max m only moves (and O, l are rescaled) when a
// tile's row max exceeds m by more than kRescaleLog2 (p <= 2^8, safe in f32 and bf16); the decision
// is wave-uniform so the rescale is a branch, not per-tile work.  The causal mask is applied on
// diagonal tiles only.  Dropout: on the packed bf16 pairs (pack_frag_keep).
constexpr float kRescaleLog2 = 8.f;

template <int I>
struct IC { static constexpr int value = I; constexpr operator int() const { return I; } };
template <int N, int I = 0, typename F>
DLTB_DEV void static_for(F&& f) {
  if constexpr (I < N) {
    f(IC<I>{});
    static_for<N, I + 1>(f);
  }
}

template <int D>
DLTB_DEV bfx8 pack_frag(const f32x16& x, int s) {      // regs 8s .. 8s+7 -> bf16 B operand
  typedef h16_t bfx2 __attribute__((ext_vector_type(2)));
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  bfx8 f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f32x2 p = {x[8 * s + 2 * j], x[8 * s + 2 * j + 1]};
    const bfx2 b = __builtin_convertvector(p, bfx2);
    f[2 * j] = b[0];
    f[2 * j + 1] = b[1];
  }
  return f;
}

// pack_frag of sub-tile N's registers 8 S .. 8 S + 7 with the dropout applied to the PACKED pairs:
// pair j = 8N + 4S + k has its keep bits at 15 - j / 31 - j (attn_mask.h mask_bit), so (mw << j)
// holds them as the sign bits of its two halves and v_perm_b32 selector 8 / 9 replicates each into
// its 16-bit half: shift + perm + and per two probabilities.
template <int N, int S, bool DROP>
DLTB_DEV bfx8 pack_frag_keep(const f32x16& x, uint32_t mw) {
  typedef h16_t bfx2 __attribute__((ext_vector_type(2)));
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  uint4 w;
  uint32_t* wp = reinterpret_cast<uint32_t*>(&w);
  static_for<4>([&](auto K) {
    constexpr int k = K;
    const f32x2 p = {x[8 * S + 2 * k], x[8 * S + 2 * k + 1]};
    uint32_t d = __builtin_bit_cast(uint32_t, __builtin_convertvector(p, bfx2));
    if constexpr (DROP) {
      constexpr int j = 8 * N + 4 * S + k;
      static_assert(mask_bit(N, 8 * S + 2 * k) == 15 - j && mask_bit(N, 8 * S + 2 * k + 1) == 31 - j,
                    "packed keep-bit layout");
      const uint32_t sh = mw << j;
      d &= __builtin_amdgcn_perm(sh, sh, 0x09090808u);
    }
    wp[k] = d;
  });
  return __builtin_bit_cast(bfx8, w);
}

// an 8-element fragment times c, rounded back to the operand format (the softmax scale folded
// into the operand held in registers: one multiply per element per wave instead of one per score)
DLTB_DEV bfx8 scale_frag(bfx8 f, float c) {
  typedef float f32x8 __attribute__((ext_vector_type(8)));
  return __builtin_convertvector(__builtin_convertvector(f, f32x8) * c, bfx8);
}

// keep ? x : y for keep bit BIT of mw: a v_bfe_i32 mask, then a bitwise select the compiler emits
// as one v_bfi_b32 / v_bitop3_b32.  Only the bfe is inline asm: x is an MFMA result, and hipcc does
// not insert the MFMA -> VALU read wait states in front of an inline-asm reader.
template <int BIT>
DLTB_DEV float keep_sel(float x, float y, uint32_t mw) {
  uint32_t k;
  asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(k) : "v"(mw), "n"(BIT));
  return __uint_as_float((k & __float_as_uint(x)) | (~k & __float_as_uint(y)));
}

DLTB_DEV f32x16 splat16(float v) {
  f32x16 r;
#pragma unroll
  for (int i = 0; i < 16; ++i) r[i] = v;
  return r;
}

// XCD-aware block order: consecutive workgroup ids land on different XCDs (round robin over 8),
// so walk the (head, query block) space with the XCD index as the slowest digit -> the query
// blocks of one head share an XCD's L2 for their K/V stream.  Causal grids visit the heaviest
// (last) query blocks first.
DLTB_DEV void block_coords(int nqb, int nbh, bool causal, int& qb, int& bh) {
  const int L = blockIdx.x, total = nqb * nbh;
#if DLTB_ATTN_LPT
  if (causal && (nbh & 7) == 0) {
    // causal grids several rounds deep: heaviest query blocks first over the WHOLE grid (greedy
    // longest-first balance), each XCD (workgroups b, b+8, ...) on nbh/8 consecutive heads (one KV
    // group's K / V in its L2 under GQA)
    const int hpx = nbh >> 3, r = L >> 3;
    bh = (L & 7) * hpx + r % hpx;
    qb = nqb - 1 - r / hpx;
    return;
  }
#endif
  int idx = L;
  if ((total & 7) == 0) idx = (L & 7) * (total >> 3) + (L >> 3);
  bh = idx / nqb;
  qb = idx % nqb;
  if (causal) qb = nqb - 1 - qb;
}

// KS = 4: 2-deep ring, 128 VGPRs without scratch for the non-causal (TinyGPT) kernels; the causal D = 64
// instantiations spill at 4 (16 / 28 B of scratch per lane without / with dropout) and run at 3 (151-152
// VGPRs, no scratch): profiles/attention_d64_resources_r5.txt
template <int D, bool C = false>
constexpr int fwd_ks() { return D == 64 ? (C && DLTB_CAUSAL_KS_CAP && DLTB_FWD_KS64 > 3 ? 3 : DLTB_FWD_KS64) : 2; }
template <int D, int KS>
constexpr int fwd_nst() {   // LDS ring depth (D = 128: 2 x 2 splits x 33 KiB)
  return D == 64 && KS < 4 ? 3 : 2;
}
template <int D>
constexpr int fwd_stage_bytes() { return 2 * kTile * D * 2 + 1024; }   // K, V, dropout words of 4 waves
template <int D, int KS = fwd_ks<D>()>
constexpr int fwd_smem_bytes() { return fwd_nst<D, KS>() * KS * fwd_stage_bytes<D>(); }

template <int D, bool CAUSAL, bool DROP, int KS>
__global__ __launch_bounds__(256 * KS) void attn_fwd_kernel(AttnArgs P) {
  constexpr int TB = kTile * D * 2;
  constexpr int NACC = D / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, h = lane >> 5;
  const int qw = w & 3, sp = w >> 2, stid = tid & 255;
  const int T = P.T, nT = T / kTile;
  int qb, bh;
  block_coords(T / kBlockRows, P.B * P.Hq, CAUSAL, qb, bh);
  const int b = bh / P.Hq, hq = bh % P.Hq, hk = hq / (P.Hq / P.Hkv);
  const int q0 = qb * kBlockRows + qw * 32;
  const int qi = q0 + r;
  DLTB_DCHECK(qi < T && bh < P.B * P.Hq && hk < P.Hkv);

  bfx8 qf[D / 16];
  {
    const bf16_t* qrow = P.q + ((long)b * T + qi) * P.q_stride + hq * D;
#pragma unroll
    for (int s = 0; s < D / 16; ++s)       // Q c: S' = (Q c) K^T is already in log2 units
      qf[s] = scale_frag(__builtin_bit_cast(bfx8, ld16<uint4>(qrow + 16 * s + 8 * h)), P.scale * kLog2e);
  }
  const int nt = CAUSAL ? min(nT, (qb * kBlockRows + kBlockRows - 1) / kTile + 1) : nT;
  const int nit = (nt + KS - 1) / KS;
  const bf16_t* kbase = P.k + (long)b * T * P.k_stride + hk * D;
  const bf16_t* vbase = P.v + (long)b * T * P.v_stride + hk * D;
  const uint32_t* mbase = DROP ? P.mask + (long)bh * nT * 2 * T : nullptr;   // wave-uniform
  const uint32_t* mrow = DROP ? mbase + (long)h * T + qi : nullptr;

  // NST-deep ring of (K, V, dropout-word) stages per key split, filled by compiler-invisible
  // LDS-DMA; a counted vmcnt retires only the stage about to be read and a raw s_barrier
  // publishes it, so NST-2 later stages stay in flight across the barrier.
  constexpr int NST = fwd_nst<D, KS>();
  constexpr int SB = fwd_stage_bytes<D>();
  constexpr int GL = 2 * GldsTile<D, kTile>::NI + (DROP ? 1 : 0);   // DMA instructions per stage
  const int wv = __builtin_amdgcn_readfirstlane(qw);
  const int spu = __builtin_amdgcn_readfirstlane(sp);      // the key split is wave-uniform
  auto stage_ptr = [&](int it) { return smem + ((it % NST) * KS + spu) * SB; };
  // per-lane DMA offsets are tile-invariant; the tile's row goes into the SGPR base (SALU only)
  uint32_t koff[GldsTile<D, kTile>::NI], voff[GldsTile<D, kTile>::NI];
  GldsTile<D, kTile>::offsets(P.k_stride, wv, lane, koff);
  GldsTile<D, kTile>::offsets(P.v_stride, wv, lane, voff);
  const uint32_t moff = (uint32_t)(mrow - mbase) * 4u;
  auto issue = [&](int it) {
    const int t = it * KS + spu;
    if (it >= nit || t >= nt) return;
    char* st = smem + ((it % NST) * KS + spu) * SB;
    GldsTile<D, kTile>::load_sv(kbase + (long)t * kTile * P.k_stride, koff, st, wv);
    GldsTile<D, kTile>::load_sv(vbase + (long)t * kTile * P.v_stride, voff, st + TB, wv);
    if (DROP) glds4_sv(mbase + (long)t * 2 * T, moff, st + 2 * TB + wv * 256);
  };
  // loop-invariant lane offsets of the LDS fragment reads (K rows per k-step, V^T per D tile/half)
  uint32_t kfo[D / 16], vfo[NACC][2];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) kfo[s] = row_lane_off<D>(r, 2 * s + h);
#pragma unroll
  for (int dt = 0; dt < NACC; ++dt)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) vfo[dt][hf] = tr_lane_off<D>(dt * 32, hf, lane);
  wait_vm<0>();        // Q fragments landed: no compiler vmcnt wait for them inside the loop
#pragma unroll
  for (int i = 0; i < NST - 1; ++i) issue(i);

  f32x16 oacc[NACC];
#pragma unroll
  for (int dt = 0; dt < NACC; ++dt) oacc[dt] = f32x16{};
  // running max m (scaled log2 units; -inf until this wave's first tile) enters the S chain as its
  // initial accumulator mv = -m, so S' = (Q c) K^T - m comes out of the MFMAs ready for exp2: the
  // softmax costs exp + add per probability, plus the packed dropout per pair
  float m = -INFINITY, l = 0.f;
  f32x16 mv = f32x16{};
  bool fresh = true;                             // wave-uniform

  // one tile's work in three phases: S' = (Q c) K^T - m into sacc; softmax (row max, lazy rescale,
  // exp2, row sums); O^T += V^T P^T with the dropout on the packed pairs
  f32x16 sacc[2];
  auto s_tile = [&](const char* kt, int kv0) {       // S' = (Q c) K^T - m, the two key halves interleaved
    const uint32_t kb = __builtin_amdgcn_readfirstlane(lds_addr(kt));
    uint32_t ka[D / 16];
#pragma unroll
    for (int s = 0; s < D / 16; ++s) ka[s] = lane_addr(kb, kfo[s]);
    sacc[0] = mfma32(row_frag_at<0>(ka[0]), qf[0], mv);
    sacc[1] = mfma32(row_frag_at<32 * D * 2>(ka[0]), qf[0], mv);
    static_for<D / 16 - 1>([&](auto S1) {
      constexpr int s = S1 + 1;
      sacc[0] = mfma32(row_frag_at<0>(ka[s]), qf[s], sacc[0]);
      sacc[1] = mfma32(row_frag_at<32 * D * 2>(ka[s]), qf[s], sacc[1]);
    });
    if (CAUSAL && kv0 + kTile - 1 > q0) {      // diagonal tile: mask keys > query
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (kv0 + 32 * n + (i & 3) + 8 * (i >> 2) + 4 * h > qi) sacc[n][i] = -INFINITY;
    }
  };
  auto row_max = [&]() {                       // this tile's row max minus m
    float mx = sacc[0][0];
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int i = (n == 0 ? 1 : 0); i < 16; ++i) mx = fmaxf(mx, sacc[n][i]);
    // the other half of the row sits in lane ^ 32: one v_permlane32_swap, no LDS round trip
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
    return fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
  };
  // move m by d = mx (first tile) or max(mx, 0): rescale l, O and this tile's S'.  Every
  // visited tile holds at least one unmasked key per row (causal: kv0 <= q0), so mx is finite.
  auto rescale = [&](float mx) {
    const float d = fresh ? mx : fmaxf(mx, 0.f);
    if (!fresh) {
      const float alpha = __builtin_amdgcn_exp2f(-d);
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < NACC; ++dt) oacc[dt] *= alpha;
    }
    m = fresh ? mx : m + d;
#pragma unroll
    for (int n = 0; n < 2; ++n) sacc[n] -= d;
    mv = splat16(-m);
    fresh = false;
  };
  auto softmax = [&]() {
    // lazy rescale: m moves only on the first tile or when a row max exceeds it by more than
    // kRescaleLog2 (p <= 2^8 in between); wave-uniform, rare after the first tiles
    {
      const float mx = row_max();
      if (fresh || __ballot(mx > kRescaleLog2)) rescale(mx);
    }
    float ls0 = 0.f, ls1 = 0.f;
    static_for<32>([&](auto J) {
      constexpr int n = J / 16, i = J % 16;
      const float p = __builtin_amdgcn_exp2f(sacc[n][i]);
      if constexpr (i & 1) ls1 += p;
      else ls0 += p;
      sacc[n][i] = p;
    });
    l += ls0 + ls1;
  };
  auto pv = [&](const char* vt, uint32_t mw) {
    const uint32_t vb = __builtin_amdgcn_readfirstlane(lds_addr(vt));
    uint32_t va[NACC][2];
#pragma unroll
    for (int dt = 0; dt < NACC; ++dt)
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) va[dt][hf] = lane_addr(vb, vfo[dt][hf]);
    static_for<4>([&](auto J) {
      constexpr int n = J / 2, s2 = J % 2;
      const bfx8 pf = pack_frag_keep<n, s2, DROP>(sacc[n], mw);
#pragma unroll
      for (int dt = 0; dt < NACC; ++dt)
        oacc[dt] = mfma32(tr_frag_at<(32 * n + 16 * s2) * D * 2>(va[dt][0], va[dt][1]), pf, oacc[dt]);
    });
  };
  auto mask_word = [&](const char* st) {
    return DROP ? *reinterpret_cast<const uint32_t*>(st + 2 * TB + wv * 256 + lane * 4) : 0u;
  };
  auto visible = [&](int t) { return t < nt && (!CAUSAL || t * kTile <= q0 + 31); };

  {
    for (int it = 0; it < nit; ++it) {
      const int t = it * KS + spu;                   // wave-uniform: the tile branches are scalar
      // stages it+1 .. it+NST-2 (issued only if their tiles exist for this split) may stay in flight
      static_assert(NST <= 4, "the counted wait below assumes at most two later stages in flight");
      const int later = NST < 3 ? 0 : min(NST - 2, min(nit - 1, (nt - 1 - spu) / KS) - it);
      if (NST > 3 && later >= 2) wait_vm<(NST > 3 ? 2 * GL : 0)>();
      else if (NST > 2 && later >= 1) wait_vm<(NST > 2 ? GL : 0)>();
      else wait_vm<0>();
      __builtin_amdgcn_s_barrier();
      issue(it + NST - 1);                         // refills the buffer read in iteration it - 1
      const char* kt = stage_ptr(it);
      if (visible(t)) {
        const uint32_t mw = mask_word(kt);
        s_tile(kt, t * kTile);
        softmax();
        pv(kt + TB, mw);
      }
    }
  }
  __syncthreads();              // all LDS reads done before the ring is reused for the merge
  if constexpr (KS > 1) {      // merge the key splits: splits 1..KS-1 -> LDS -> split 0
    constexpr int NF = 16 * NACC + 2;
    static_assert((KS - 1) * 4 * NF * 64 * 4 <= NST * KS * SB, "merge buffer exceeds the LDS ring");
    float* red0 = reinterpret_cast<float*>(smem) + qw * NF * 64 + lane;
    if (sp > 0) {
      float* red = red0 + (sp - 1) * 4 * NF * 64;
      red[0] = m;
      red[64] = l;
#pragma unroll
      for (int dt = 0; dt < NACC; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) red[(2 + 16 * dt + i) * 64] = oacc[dt][i];
    }
    __syncthreads();
    if (sp > 0) return;
#pragma unroll
    for (int o = 0; o < KS - 1; ++o) {
      const float* red = red0 + o * 4 * NF * 64;
      const float m1 = red[0], l1 = red[64];
      const float mn = fmaxf(m, m1);
      const float a0 = __builtin_amdgcn_exp2f(m - mn), a1 = __builtin_amdgcn_exp2f(m1 - mn);
      m = mn;
      l = l * a0 + l1 * a1;
#pragma unroll
      for (int dt = 0; dt < NACC; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) oacc[dt][i] = oacc[dt][i] * a0 + red[(2 + 16 * dt + i) * 64] * a1;
    }
  }
  l += __shfl_xor(l, 32, 64);
  const float inv = (DROP ? P.drop_scale : 1.f) / l;
  bf16_t* orow = P.out + ((long)b * T + qi) * P.out_stride + hq * D;
  store_acc_rows<D>(orow, oacc, inv, h);
  if (h == 0) P.lse[((long)b * P.Hq + hq) * T + qi] = (m + __log2f(l)) * 0.69314718055994531f;
}



// =============================================================================== backward prep
// delta[b, h, t] = sum_d dO[b,t,h,d] * O[b,t,h,d]
template <int D>
__global__ __launch_bounds__(256) void attn_bwd_delta_kernel(AttnArgs P) {
  constexpr int CH = D / 8;
  const long gid = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const long row = gid / CH;               // (b, t, h) in token-major order
  const int ch = (int)(gid % CH);
  const long total = (long)P.B * P.T * P.Hq;
  float acc = 0.f;
  long bt = 0;
  int hq = 0;
  if (row < total) {
    bt = row / P.Hq;
    hq = (int)(row % P.Hq);
    float a[8], o[8];
    unpack8(ld16<uint4>(P.dout + bt * P.do_stride + hq * D + ch * 8), a);
    unpack8(ld16<uint4>(P.o + bt * P.o_stride + hq * D + ch * 8), o);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc += a[e] * o[e];
  }
#pragma unroll
  for (int off = CH / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if (row < total && ch == 0) {
    const long b = bt / P.T, t = bt % P.T;
    const_cast<float*>(P.delta)[(b * P.Hq + hq) * P.T + t] = acc;
  }
}

// =============================================================================== dK / dV
// Workgroup = KS query-splits x 4 waves; wave (kw, sp) owns keys k0 .. k0+31 (K, V in registers)
// and sweeps the query tiles t == sp (mod KS) of every query head of its KV group.  The two
// partial dK/dV accumulators merge through LDS at the end.  Dropout folds into
//   pd = p & keep,  ds' = p * ((dp & keep) - delta / s)     (s = 1/(1-p); dK, dV scaled by s at the store)
// so each probability costs bfe + 2 and + sub + mul besides its exp.
#ifndef DLTB_DKDV_KS64
#define DLTB_DKDV_KS64 2   // query splits per dK/dV workgroup at D = 64; 3 (168 VGPRs, 80 B scratch) is 25 % slower
                           // (profiles/attention_dkdv_ks3_ab_r4.txt)
#endif
template <int D>
constexpr int dkdv_ks() { return D == 64 ? DLTB_DKDV_KS64 : 1; }
// dropout words in LDS: [4 subs][kTile rows] with a 4-word pad per sub, so the two subs a wave
// reads together (lanes with key bit 2 clear / set) and the 4 subs one store instruction writes
// start 68 words apart -- different banks, where an unpadded 64-word stride put them all on the
// same bank (the 12 % LDS bank conflicts of profiles/attention_pmc_tinygpt_a.txt)
constexpr int kMaskStride = kTile + 4;
template <int D>
constexpr int dkdv_stage_bytes() { return 2 * kTile * D * 2 + 2 * kTile * 4 + 4 * kMaskStride * 4; }
template <int D>
constexpr int dkdv_smem_bytes() {
  constexpr int a = 2 * dkdv_ks<D>() * dkdv_stage_bytes<D>();
  constexpr int merge = (dkdv_ks<D>() - 1) * 4 * 64 * 4 * (2 * 16 * (D / 32));
  return merge > a ? merge : a;
}

DLTB_DEV uint32_t keep_mask_v(uint32_t mw, uint32_t bit) {
  uint32_t k;
  asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(k) : "v"(mw), "v"(bit));
  return k;
}

// splits 1..KS-1 -> LDS -> split 0, then the scaled bf16 (or fp32 head-split partial) stores of split 0.
// The caller guarantees no wave still reads the tile stages (the merge reuses the LDS from offset 0).
template <int D, int KS, bool DROP>
DLTB_DEV void dkdv_finish(const AttnArgs& P, char* smem, f32x16 (&dk)[D / 32], f32x16 (&dv)[D / 32], int kw,
                          int sp, int lane, int h, int b, int hk, int key, int gs) {
  constexpr int NACC = D / 32;
  const int T = P.T;
  if constexpr (KS > 1) {
    constexpr int NF = 2 * 16 * NACC;
    float* red0 = reinterpret_cast<float*>(smem) + kw * NF * 64 + lane;
    if (sp > 0) {
      float* red = red0 + (sp - 1) * 4 * NF * 64;
#pragma unroll
      for (int dt = 0; dt < NACC; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          red[(16 * dt + i) * 64] = dk[dt][i];
          red[(16 * (NACC + dt) + i) * 64] = dv[dt][i];
        }
    }
    __syncthreads();
    if (sp > 0) return;
#pragma unroll
    for (int o = 0; o < KS - 1; ++o)
#pragma unroll
      for (int dt = 0; dt < NACC; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          dk[dt][i] += red0[o * 4 * NF * 64 + (16 * dt + i) * 64];
          dv[dt][i] += red0[o * 4 * NF * 64 + (16 * (NACC + dt) + i) * 64];
        }
  }
  const float s_drop = DROP ? P.drop_scale : 1.f;
  if (P.gsplit > 1) {      // partial over this workgroup's heads -> fp32, summed by dkdv_reduce_kernel
    const long plane = (long)P.B * T * P.Hkv * D;
    float* pk = P.part + 2 * gs * plane + ((long)b * T + key) * P.Hkv * D + hk * D;
    store_acc_rows_f32<D>(pk, dk, P.scale * s_drop, h);
    store_acc_rows_f32<D>(pk + plane, dv, s_drop, h);
    return;
  }
  bf16_t* dkrow = P.out + ((long)b * T + key) * P.out_stride + hk * D;
  bf16_t* dvrow = P.out2 + ((long)b * T + key) * P.out2_stride + hk * D;
  store_acc_rows<D>(dkrow, dk, P.scale * s_drop, h);
  store_acc_rows<D>(dvrow, dv, s_drop, h);
}

template <int D, bool CAUSAL, bool DROP, int KS>
__global__ __launch_bounds__(256 * KS) void attn_bwd_dkdv_kernel(AttnArgs P) {
  constexpr int TB = kTile * D * 2;
  constexpr int SB = dkdv_stage_bytes<D>();   // Q tile, dO tile, lse2[64], delta'[64], mask[64][4]
  constexpr int NACC = D / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, h = lane >> 5;
  const int kw = w & 3, sp = w >> 2, stid = tid & 255;
  const int T = P.T, nT = T / kTile;
  int kb, bk;
  const int gsplit = P.gsplit;
  if (CAUSAL && gsplit > 1) {
    // head-split causal grids: key block (the work: query tiles kb*2 .. nT-1) is the SLOW index, so
    // the grid is dispatched heaviest first over all heads and the workgroups that free their slot
    // early pick up the light blocks (greedy longest-first balance).  The (head, split) index is
    // fast: with nbk % 8 == 0 the workgroups of one XCD (b, b+8, ...) cover nbk/8 of them and share
    // their Q / dO tiles in its L2.  (block_coords' XCD remap cycled kb 0..nkb-1 once per 8 x nkb
    // workgroups, so heavy blocks kept arriving until the end of the grid.)
    // (pairing key blocks kb and nkb-1-kb across the two halves of the grid measured 18 % slower:
    // profiles/dkdv_lpt_map_m7b_r3.txt)
    const int nbk = P.B * P.Hkv * gsplit;
    kb = blockIdx.x / nbk;
    bk = blockIdx.x - kb * nbk;
  } else {
    block_coords(T / kBlockRows, P.B * P.Hkv * gsplit, false, kb, bk);
  }
  const int gs = bk % gsplit;
  bk /= gsplit;
  // one workgroup per key block and KV head: all resident at once, heaviest (first keys) last
  if (CAUSAL && gsplit == 1) kb = T / kBlockRows - 1 - kb;
  const int b = bk / P.Hkv, hk = bk % P.Hkv;
  const int G = P.Hq / P.Hkv / gsplit, g0 = gs * G;   // this workgroup's query heads of the group
  const int kblk0 = kb * kBlockRows;
  const int k0 = kblk0 + kw * 32;
  const int key = k0 + r;
  // this lane's bit in the packed mask words (see attn_mask_kernel)
  const int hbit = (r >> 2) & 1;
  const uint32_t jbit = mask_bit(kw & 1, (r & 3) | (((r >> 3) & 3) << 2));
  const int msub = (kw >> 1) * 2 + hbit;
  const float inv_s = DROP ? 1.f / P.drop_scale : 1.f;

  bfx8 kf[D / 16], vf[D / 16];
  {
    const bf16_t* krow = P.k + ((long)b * T + key) * P.k_stride + hk * D;
    const bf16_t* vrow = P.v + ((long)b * T + key) * P.v_stride + hk * D;
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      // K c: S' = Q (K c)^T - lse log2(e) is the exp2 argument itself (no multiply per score)
      kf[s] = scale_frag(__builtin_bit_cast(bfx8, ld16<uint4>(krow + 16 * s + 8 * h)), P.scale * kLog2e);
      vf[s] = __builtin_bit_cast(bfx8, ld16<uint4>(vrow + 16 * s + 8 * h));
    }
  }
  f32x16 dk[NACC], dv[NACC];
#pragma unroll
  for (int dt = 0; dt < NACC; ++dt) { dk[dt] = f32x16{}; dv[dt] = f32x16{}; }

  const int t_begin = CAUSAL ? kblk0 / kTile : 0;
  const int nit = (nT - t_begin + KS - 1) / KS;   // iterations per head
  const int njobs = G * nit;

  const int wv = __builtin_amdgcn_readfirstlane(kw);
  float vl = 0.f, vd = 0.f;
  uint32_t mword = 0;
  const int spu = __builtin_amdgcn_readfirstlane(sp);   // wave-uniform: tile math stays in SGPRs
  auto tile_of = [&](int j, int& g, int& t) { g = g0 + j / nit; t = t_begin + (j % nit) * KS + spu; };
  // loop-invariant per-lane parts of every streamed address (the Q / dO LDS-DMA offsets, the
  // dropout-word offset); per tile only wave-uniform (SGPR) bases change -- no per-tile VALU
  // address arithmetic (64-bit multiplies) in the loop
  uint32_t qoff[GldsTile<D, kTile>::NI], doff[GldsTile<D, kTile>::NI];
  GldsTile<D, kTile>::offsets(P.q_stride, wv, lane, qoff);
  GldsTile<D, kTile>::offsets(P.do_stride, wv, lane, doff);
  const int mrow = stid >> 2, msb = stid & 3;
  const uint32_t moff = (uint32_t)(msb * T + mrow);    // ((.. + (sb >> 1)) * 2 + (sb & 1)) * T + row
  auto load = [&](int j) {
    int g, t;
    tile_of(j, g, t);
    if (t >= nT) return;
    const int hq = hk * G * gsplit + g;
    const long bq = (long)b * P.Hq + hq;
    // Q / dO tiles straight into the stage buffer by LDS-DMA (it is not being read: the previous
    // reader of this buffer finished before the last barrier)
    char* base = smem + ((j & 1) * KS + sp) * SB;
    const long r0 = (long)b * T + t * kTile;
    GldsTile<D, kTile>::load_sv(P.q + r0 * P.q_stride + hq * D, qoff, base, wv);
    GldsTile<D, kTile>::load_sv(P.dout + r0 * P.do_stride + hq * D, doff, base + TB, wv);
    if (stid < kTile) {   // row constants, loaded straight into the S / dP accumulators
      const long rc = bq * T + t * kTile;
      vl = -P.lse[rc + stid] * kLog2e;
      vd = -P.delta[rc + stid] * inv_s;
    }
    if (DROP) mword = P.mask[((bq * nT + kb * 2) * 2) * T + t * kTile + moff];
  };
  auto store = [&](int j) {
    int g, t;
    tile_of(j, g, t);
    if (t >= nT) return;
    char* base = smem + ((j & 1) * KS + sp) * SB;
    float* f = reinterpret_cast<float*>(base + 2 * TB);
    if (stid < kTile) {
      f[stid] = vl;
      f[kTile + stid] = vd;
    }
    if (DROP)     // [sub][row]: a lane's 4 consecutive query rows are one ds_read_b128
      reinterpret_cast<uint32_t*>(f + 2 * kTile)[msb * kMaskStride + mrow] = mword;
  };
  load(0);
  store(0);
  wait_vm<0>();        // this wave's LDS-DMA share landed (the compiler does not track the asm DMA)
  __syncthreads();
  for (int j = 0; j < njobs; ++j) {
    int g_, t;
    tile_of(j, g_, t);
    const char* qt = smem + ((j & 1) * KS + sp) * SB;
    const char* dt_ = qt + TB;
    const float* lse2 = reinterpret_cast<const float*>(qt + 2 * TB);
    const float* dlt = lse2 + kTile;
    const uint32_t* mws = reinterpret_cast<const uint32_t*>(dlt + kTile);
    if (j + 1 < njobs) load(j + 1);
    // S' = Q (K c)^T - lse log2(e) and dP' = dO V^T - delta/s: p = exp2(S'), ds = p dP' (no dropout)
    auto sdp = [&](int mm, f32x16& sa, f32x16& dp) {
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int ql = 32 * mm + 8 * g4 + 4 * h;
        const float4 L = *reinterpret_cast<const float4*>(lse2 + ql);
        sa[4 * g4 + 0] = L.x; sa[4 * g4 + 1] = L.y; sa[4 * g4 + 2] = L.z; sa[4 * g4 + 3] = L.w;
        if (DROP) {
          dp[4 * g4 + 0] = 0.f; dp[4 * g4 + 1] = 0.f; dp[4 * g4 + 2] = 0.f; dp[4 * g4 + 3] = 0.f;
        } else {
          const float4 Dl = *reinterpret_cast<const float4*>(dlt + ql);
          dp[4 * g4 + 0] = Dl.x; dp[4 * g4 + 1] = Dl.y; dp[4 * g4 + 2] = Dl.z; dp[4 * g4 + 3] = Dl.w;
        }
      }
      if constexpr (D == 128) {        // 1 wave / SIMD: all fragments first (one lgkmcnt wait)
        bfx8 qa[D / 16], da[D / 16];
#pragma unroll
        for (int s = 0; s < D / 16; ++s) {
          qa[s] = row_frag<D>(qt, 32 * mm + r, 2 * s + h);
          da[s] = row_frag<D>(dt_, 32 * mm + r, 2 * s + h);
        }
#pragma unroll
        for (int s = 0; s < D / 16; ++s) {
          sa = mfma32(qa[s], kf[s], sa);
          dp = mfma32(da[s], vf[s], dp);
        }
      } else {                         // several waves / SIMD hide the reads; keep registers low
#pragma unroll
        for (int s = 0; s < D / 16; ++s) {
          sa = mfma32(row_frag<D>(qt, 32 * mm + r, 2 * s + h), kf[s], sa);
          dp = mfma32(row_frag<D>(dt_, 32 * mm + r, 2 * s + h), vf[s], dp);
        }
      }
    };
    auto softmax = [&](int mm, const f32x16& sa, const f32x16& dp, bool diag, f32x16& pd, f32x16& ds) {
      const int qb = t * kTile + 32 * mm;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int ql = 32 * mm + 8 * g4 + 4 * h;
        float4 Dl;
        uint4 M4;
        if (DROP) {
          Dl = *reinterpret_cast<const float4*>(dlt + ql);
          M4 = *reinterpret_cast<const uint4*>(mws + msub * kMaskStride + ql);
        }
        const float Dv[4] = {Dl.x, Dl.y, Dl.z, Dl.w};
        const uint32_t Mv[4] = {M4.x, M4.y, M4.z, M4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 4 * g4 + e;
          float p = __builtin_amdgcn_exp2f(sa[i]);
          if (CAUSAL && diag && key > qb + 8 * g4 + 4 * h + e) p = 0.f;
          if (DROP) {     // dS = fma(p keep, dP', p D): the masked probability carries the keep bit
            const float pdv = __uint_as_float(__float_as_uint(p) & keep_mask_v(Mv[e], jbit));
            pd[i] = pdv;
            ds[i] = __builtin_fmaf(pdv, dp[i], p * Dv[e]);
          } else {
            pd[i] = p;
            ds[i] = p * dp[i];
          }
        }
      }
    };
    auto accum = [&](int mm, const f32x16& pd, const f32x16& ds) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bfx8 pf = pack_frag<D>(pd, s2);
        const bfx8 sf = pack_frag<D>(ds, s2);
#pragma unroll
        for (int d_ = 0; d_ < NACC; ++d_) {
          dv[d_] = mfma32(tr_frag<D>(dt_, 32 * mm + 16 * s2, d_ * 32, lane), pf, dv[d_]);
          dk[d_] = mfma32(tr_frag<D>(qt, 32 * mm + 16 * s2, d_ * 32, lane), sf, dk[d_]);
        }
      }
    };
    if (t < nT) {
      if (D == 128 && (!CAUSAL || t * kTile >= k0 + 31)) {
        // full tile (no mask): both sub-tiles' S/dP first, so the second pair's MFMAs overlap the
        // first sub-tile's softmax, and its dV/dK MFMAs overlap the second softmax
        f32x16 sa0, dp0, sa1, dp1, pd, ds;
        sdp(0, sa0, dp0);
        sdp(1, sa1, dp1);
        softmax(0, sa0, dp0, false, pd, ds);
        accum(0, pd, ds);
        softmax(1, sa1, dp1, false, pd, ds);
        accum(1, pd, ds);
      } else {
#pragma unroll
        for (int mm = 0; mm < 2; ++mm) {
          const int qb = t * kTile + 32 * mm;
          if (CAUSAL && qb + 31 < k0) continue;   // every query < every key of this wave
          f32x16 sa, dp, pd, ds;
          sdp(mm, sa, dp);
          softmax(mm, sa, dp, qb < k0 + 31, pd, ds);
          accum(mm, pd, ds);
        }
      }
    }
    if (j + 1 < njobs) store(j + 1);
    wait_vm<0>();
    __syncthreads();
  }
  dkdv_finish<D, KS, DROP>(P, smem, dk, dv, kw, sp, lane, h, b, hk, key, gs);
}

// dK / dV = sum of the head-split partials (8 columns per thread), bf16 into the strided outputs
__global__ __launch_bounds__(256) void dkdv_reduce_kernel(const float* __restrict__ part, int gsplit,
                                                          long rows, int cols, bf16_t* __restrict__ dk,
                                                          long dks, bf16_t* __restrict__ dv, long dvs) {
  const long plane = rows * cols;
  const long i = ((long)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i >= 2 * plane) return;
  const int which = i >= plane;
  const long e = i - which * plane;
  float a[8];
  {
    const float4 x0 = *reinterpret_cast<const float4*>(part + i);
    const float4 x1 = *reinterpret_cast<const float4*>(part + i + 4);
    a[0] = x0.x; a[1] = x0.y; a[2] = x0.z; a[3] = x0.w; a[4] = x1.x; a[5] = x1.y; a[6] = x1.z; a[7] = x1.w;
  }
  for (int s = 1; s < gsplit; ++s) {
    const float* src = part + 2 * s * plane + i;
    const float4 x0 = *reinterpret_cast<const float4*>(src);
    const float4 x1 = *reinterpret_cast<const float4*>(src + 4);
    a[0] += x0.x; a[1] += x0.y; a[2] += x0.z; a[3] += x0.w;
    a[4] += x1.x; a[5] += x1.y; a[6] += x1.z; a[7] += x1.w;
  }
  const long r = e / cols, c = e % cols;
  bf16_t* dst = which ? dv + r * dvs + c : dk + r * dks + c;
  uint4 o;
  o.x = pack_bf2(a[0], a[1]);
  o.y = pack_bf2(a[2], a[3]);
  o.z = pack_bf2(a[4], a[5]);
  o.w = pack_bf2(a[6], a[7]);
  *reinterpret_cast<uint4*>(dst) = o;
}

// =============================================================================== dQ
// Query-major, KS key-splits per workgroup as in the forward; dQ partials merge through LDS.
// causal D = 64 with dropout spills at 3 (40 B of scratch per lane): 2 splits there (188 VGPRs, no scratch)
template <int D, bool C = false>
constexpr int dq_ks() { return D == 64 ? (C && DLTB_CAUSAL_KS_CAP && DLTB_DQ_KS64 > 2 ? 2 : DLTB_DQ_KS64) : 2; }
template <int D>
constexpr int dq_nst() { return D == 64 ? 3 : 2; }   // LDS ring depth, as the forward's
template <int D>
constexpr int dq_stage_bytes() { return 2 * kTile * D * 2 + 1024; }   // K, V, dropout words of 4 waves
template <int D, int KS = dq_ks<D>()>
constexpr int dq_smem_bytes() {
  constexpr int ring = dq_nst<D>() * KS * dq_stage_bytes<D>();
  constexpr int merge = (KS - 1) * 4 * 16 * (D / 32) * 64 * 4;
  return ring > merge ? ring : merge;
}

template <int D, bool CAUSAL, bool DROP, int KS>
__global__ __launch_bounds__(256 * KS) void attn_bwd_dq_kernel(AttnArgs P) {
  constexpr int TB = kTile * D * 2;
  constexpr int NACC = D / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, h = lane >> 5;
  const int qw = w & 3, sp = w >> 2, stid = tid & 255;
  const int T = P.T, nT = T / kTile;
  int qb, bh;
  block_coords(T / kBlockRows, P.B * P.Hq, CAUSAL, qb, bh);
  const int b = bh / P.Hq, hq = bh % P.Hq, hk = hq / (P.Hq / P.Hkv);
  const int q0 = qb * kBlockRows + qw * 32;
  const int qi = q0 + r;
  const long bq = (long)b * P.Hq + hq;

  bfx8 qf[D / 16], of[D / 16];
  {
    const bf16_t* qrow = P.q + ((long)b * T + qi) * P.q_stride + hq * D;
    const bf16_t* dorow = P.dout + ((long)b * T + qi) * P.do_stride + hq * D;
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      qf[s] = __builtin_bit_cast(bfx8, ld16<uint4>(qrow + 16 * s + 8 * h));
      of[s] = __builtin_bit_cast(bfx8, ld16<uint4>(dorow + 16 * s + 8 * h));
    }
  }
  float dlt;
  if (P.o) {   // fused delta = rowsum(dO * O) for this row (replaces attn_bwd_delta_kernel)
    // summed in attn_bwd_delta_kernel's order (8-element chunks, then its xor butterfly over the
    // chunks; this lane holds chunks 2s + h), so both paths give bitwise the same delta
    const bf16_t* orow = P.o + ((long)b * T + qi) * P.o_stride + hq * D;
    constexpr int NS = D / 16;
    float cs[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      float a[8], c[8];
      unpack8(ld16<uint4>(orow + 16 * s + 8 * h), a);
      unpack8(__builtin_bit_cast(uint4, of[s]), c);
      float acc = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc += c[e] * a[e];
      cs[s] = acc;
    }
#pragma unroll
    for (int off = NS / 2; off > 0; off >>= 1)
#pragma unroll
      for (int s = 0; s < off; ++s) cs[s] += cs[s + off];
    dlt = cs[0] + __shfl_xor(cs[0], 32, 64);
    if (sp == 0 && h == 0) const_cast<float*>(P.delta)[bq * T + qi] = dlt;   // read by dK/dV next
  } else {
    dlt = P.delta[bq * T + qi];
  }
  // row constants as the initial accumulators: S' = (Q c) K^T - lse log2(e) is the exp2 argument
  // and dP' = dO V^T - delta/s, so p = exp2(S'), dS = p (keep ? dP' : -delta/s)
  const f32x16 nlv = splat16(-P.lse[bq * T + qi] * kLog2e);
  const float nd = -dlt * (DROP ? 1.f / P.drop_scale : 1.f);
  const f32x16 ndv = splat16(nd);
#pragma unroll
  for (int s = 0; s < D / 16; ++s) qf[s] = scale_frag(qf[s], P.scale * kLog2e);   // after the delta dot
  const uint32_t* mbase = DROP ? P.mask + (long)bq * nT * 2 * T : nullptr;   // wave-uniform
  const uint32_t* mrow = DROP ? mbase + (long)h * T + qi : nullptr;
  const int nt = CAUSAL ? min(nT, (qb * kBlockRows + kBlockRows - 1) / kTile + 1) : nT;
  const int nit = (nt + KS - 1) / KS;
  const bf16_t* kbase = P.k + (long)b * T * P.k_stride + hk * D;
  const bf16_t* vbase = P.v + (long)b * T * P.v_stride + hk * D;

  // NST-deep ring of (K, V, dropout-word) stages per key split, filled by compiler-invisible
  // LDS-DMA (the forward's scheme): a counted vmcnt retires only the stage about to be read and a
  // raw s_barrier publishes it, so later stages stay in flight across the barrier.
  constexpr int NST = dq_nst<D>();
  constexpr int SB = dq_stage_bytes<D>();
  constexpr int GL = 2 * GldsTile<D, kTile>::NI + (DROP ? 1 : 0);   // DMA instructions per stage
  const int wv = __builtin_amdgcn_readfirstlane(qw);
  auto stage_ptr = [&](int it) { return smem + ((it % NST) * KS + sp) * SB; };
  // per-lane DMA offsets are tile-invariant; the tile's row goes into the SGPR base (SALU only)
  uint32_t koff[GldsTile<D, kTile>::NI], voff[GldsTile<D, kTile>::NI];
  GldsTile<D, kTile>::offsets(P.k_stride, wv, lane, koff);
  GldsTile<D, kTile>::offsets(P.v_stride, wv, lane, voff);
  const uint32_t moff = (uint32_t)(mrow - mbase) * 4u;
  const int spu = __builtin_amdgcn_readfirstlane(sp);      // the key split is wave-uniform
  auto issue = [&](int it) {
    const int t = it * KS + spu;
    if (it >= nit || t >= nt) return;
    char* st = smem + ((it % NST) * KS + spu) * SB;
    GldsTile<D, kTile>::load_sv(kbase + (long)t * kTile * P.k_stride, koff, st, wv);
    GldsTile<D, kTile>::load_sv(vbase + (long)t * kTile * P.v_stride, voff, st + TB, wv);
    if (DROP) glds4_sv(mbase + (long)t * 2 * T, moff, st + 2 * TB + wv * 256);
  };
  wait_vm<0>();        // Q / dO (/ O) fragments and the delta store done: no compiler wait in the loop
#pragma unroll
  for (int i = 0; i < NST - 1; ++i) issue(i);

  f32x16 dq[NACC];
#pragma unroll
  for (int dt = 0; dt < NACC; ++dt) dq[dt] = f32x16{};

  for (int it = 0; it < nit; ++it) {
    const int t = it * KS + sp;
    static_assert(NST <= 3, "the counted wait below assumes at most one later stage in flight");
    if (NST > 2 && it + 1 < nit && (it + 1) * KS + sp < nt) wait_vm<(NST > 2 ? GL : 0)>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    issue(it + NST - 1);                         // refills the buffer read in iteration it - 1
    const char* kt = stage_ptr(it);
    const char* vt = kt + TB;
    const uint32_t mw = DROP ? *reinterpret_cast<const uint32_t*>(kt + 2 * TB + wv * 256 + lane * 4) : 0u;
    const int kv0 = t * kTile;
    // S^T / dP^T of key sub-tile n (32 keys x this wave's 32 queries)
    auto sdp = [&](int n, f32x16& sa, f32x16& dp) {
      sa = nlv;
      dp = ndv;
#pragma unroll
      for (int s = 0; s < D / 16; ++s) {
        sa = mfma32(row_frag<D>(kt, 32 * n + r, 2 * s + h), qf[s], sa);
        dp = mfma32(row_frag<D>(vt, 32 * n + r, 2 * s + h), of[s], dp);
      }
    };
    // softmax / dS of sub-tile n and dQ^T += K^T dS^T
    auto fin = [&](int n, const f32x16& sa, const f32x16& dp) {
      const bool diag = CAUSAL && kv0 + 32 * n + 31 > q0;
      f32x16 ds;
      static_for<16>([&](auto I) {
        constexpr int i = I;
        float p = __builtin_amdgcn_exp2f(sa[i]);
        if (diag && kv0 + 32 * n + (i & 3) + 8 * (i >> 2) + 4 * h > qi) p = 0.f;
        const float dpv = DROP ? (n == 0 ? keep_sel<mask_bit(0, i)>(dp[i], nd, mw)
                                         : keep_sel<mask_bit(1, i)>(dp[i], nd, mw)) : dp[i];
        ds[i] = p * dpv;
      });
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bfx8 sf = pack_frag<D>(ds, s2);
#pragma unroll
        for (int dt = 0; dt < NACC; ++dt)
          dq[dt] = mfma32(tr_frag<D>(kt, 32 * n + 16 * s2, dt * 32, lane), sf, dq[dt]);
      }
    };
    if (t < nt) {
      {
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          if (CAUSAL && kv0 + 32 * n > q0 + 31) continue;
          f32x16 sa, dp;
          sdp(n, sa, dp);
          fin(n, sa, dp);
        }
      }
    }
  }
  __syncthreads();              // all LDS reads done before the ring is reused for the merge
  if constexpr (KS > 1) {      // splits 1..KS-1 -> LDS -> split 0
    constexpr int NF = 16 * NACC;
    static_assert((KS - 1) * 4 * NF * 64 * 4 <= dq_smem_bytes<D, KS>(), "merge buffer exceeds the LDS ring");
    float* red0 = reinterpret_cast<float*>(smem) + qw * NF * 64 + lane;
    if (sp > 0) {
      float* red = red0 + (sp - 1) * 4 * NF * 64;
#pragma unroll
      for (int dt = 0; dt < NACC; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) red[(16 * dt + i) * 64] = dq[dt][i];
    }
    __syncthreads();
    if (sp > 0) return;
#pragma unroll
    for (int o = 0; o < KS - 1; ++o)
#pragma unroll
      for (int dt = 0; dt < NACC; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) dq[dt][i] += red0[o * 4 * NF * 64 + (16 * dt + i) * 64];
  }
  bf16_t* dqrow = P.out + ((long)b * T + qi) * P.out_stride + hq * D;
  store_acc_rows<D>(dqrow, dq, P.scale * (DROP ? P.drop_scale : 1.f), h);
}

AttnArgs make_args(const void* q, const void* k, const void* v, long qs, long ks, long vs, int B,
                   int T, int Hq, int Hkv, float scale, int causal, uint32_t thr16,
                   float drop_scale, const int64_t* seed, int64_t site) {
  AttnArgs a{};
  a.q = (const bf16_t*)q;
  a.k = (const bf16_t*)k;
  a.v = (const bf16_t*)v;
  a.q_stride = qs;
  a.k_stride = ks;
  a.v_stride = vs;
  a.B = B;
  a.T = T;
  a.Hq = Hq;
  a.Hkv = Hkv;
  a.scale = scale;
  a.causal = causal;
  a.thr16 = thr16;
  a.drop_scale = drop_scale;
  a.seed_ptr = seed;
  a.site = site;
  a.gsplit = 1;
  return a;
}

}  // namespace

bool dltb_attn_supported(int D, int T) { return (D == 64 || D == 128) && T % kBlockRows == 0; }

long dltb_attn_mask_words(int B, int Hq, int T) { return (long)B * Hq * (T / kTile) * 2 * T; }

namespace {

template <int D, bool C, bool DR>
void set_attrs() {
  (void)hipFuncSetAttribute((const void*)attn_fwd_kernel<D, C, DR, fwd_ks<D, C>()>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, fwd_smem_bytes<D, fwd_ks<D, C>()>());
  (void)hipFuncSetAttribute((const void*)attn_bwd_dq_kernel<D, C, DR, dq_ks<D, C>()>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, dq_smem_bytes<D, dq_ks<D, C>()>());
  if constexpr (D == 64 && C && DLTB_CAUSAL_KS_CAP && DLTB_DQ_KS64 > dq_ks<D, C>())
    (void)hipFuncSetAttribute((const void*)attn_bwd_dq_kernel<D, C, DR, DLTB_DQ_KS64>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, dq_smem_bytes<D, DLTB_DQ_KS64>());
  (void)hipFuncSetAttribute((const void*)attn_bwd_dkdv_kernel<D, C, DR, dkdv_ks<D>()>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, dkdv_smem_bytes<D>());
}

template <int D, bool C, bool DR>
void launch_fwd(const AttnArgs& a, hipStream_t st) {
  constexpr int KS = fwd_ks<D, C>();
  constexpr int smem = fwd_smem_bytes<D, KS>();
  dim3 grid((a.T / kBlockRows) * a.B * a.Hq);
  hipLaunchKernelGGL((attn_fwd_kernel<D, C, DR, KS>), grid, dim3(256 * KS), smem, st, a);
}

#define DLTB_ATTN_DISPATCH(FN, D, C, DR, ...)           \
  do {                                                  \
    if (D == 64) {                                      \
      if (C) { if (DR) FN<64, true, true>(__VA_ARGS__); else FN<64, true, false>(__VA_ARGS__); } \
      else   { if (DR) FN<64, false, true>(__VA_ARGS__); else FN<64, false, false>(__VA_ARGS__); } \
    } else {                                            \
      if (C) { if (DR) FN<128, true, true>(__VA_ARGS__); else FN<128, true, false>(__VA_ARGS__); } \
      else   { if (DR) FN<128, false, true>(__VA_ARGS__); else FN<128, false, false>(__VA_ARGS__); } \
    }                                                   \
  } while (0)

}  // namespace

void dltb_attn_init_attributes() {
  static bool done = false;
  if (done) return;
  done = true;
  set_attrs<64, false, false>();
  set_attrs<64, false, true>();
  set_attrs<64, true, false>();
  set_attrs<64, true, true>();
  set_attrs<128, false, false>();
  set_attrs<128, false, true>();
  set_attrs<128, true, false>();
  set_attrs<128, true, true>();
}

void dltb_attn_mask(uint32_t* mask, int B, int T, int Hq, uint32_t thr16, const int64_t* seed,
                    int64_t site, hipStream_t st) {
  const dim3 grid(cdiv(T, 256), (unsigned)(B * Hq * (T / kTile) * 2));
  hipLaunchKernelGGL(attn_mask_kernel, grid, dim3(256), 0, st, mask, T, thr16, seed, site);
}

void dltb_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse,
                   const uint32_t* mask, long qs, long ks, long vs, long os, int B, int T, int Hq,
                   int Hkv, int D, float scale, int causal, uint32_t thr16, float drop_scale,
                   hipStream_t st) {
  AttnArgs a = make_args(q, k, v, qs, ks, vs, B, T, Hq, Hkv, scale, causal, thr16, drop_scale,
                         nullptr, 0);
  a.out = (bf16_t*)o;
  a.out_stride = os;
  a.lse = lse;
  a.mask = mask;
  DLTB_ATTN_DISPATCH(launch_fwd, D, causal != 0, thr16 != 0, a, st);
}

void dltb_attn_bwd_delta(const void* o, const void* dout, float* delta, long os, long dos, int B,
                         int T, int Hq, int D, hipStream_t st) {
  AttnArgs a{};
  a.o = (const bf16_t*)o;
  a.o_stride = os;
  a.dout = (const bf16_t*)dout;
  a.do_stride = dos;
  a.delta = delta;
  a.B = B;
  a.T = T;
  a.Hq = Hq;
  const long rows = (long)B * T * Hq * (D / 8);
  if (D == 64)
    hipLaunchKernelGGL(attn_bwd_delta_kernel<64>, dim3(cdiv(rows, 256)), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(attn_bwd_delta_kernel<128>, dim3(cdiv(rows, 256)), dim3(256), 0, st, a);
}

namespace {
template <int D, bool C, bool DR>
void launch_dkdv(const AttnArgs& a, hipStream_t st) {
  constexpr int KS = dkdv_ks<D>();

  hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, C, DR, KS>), dim3((a.T / kBlockRows) * a.B * a.Hkv * a.gsplit),
                     dim3(256 * KS), dkdv_smem_bytes<D>(), st, a);
  if (a.gsplit > 1) {
    const long rows = (long)a.B * a.T;
    const int cols = a.Hkv * D;
    hipLaunchKernelGGL(dkdv_reduce_kernel, dim3(cdiv(2 * rows * cols / 8, 256)), dim3(256), 0, st,
                       a.part, a.gsplit, rows, cols, a.out, a.out_stride, a.out2, a.out2_stride);
  }
}
template <int D, bool C, bool DR, int KS>
void launch_dq_ks(const AttnArgs& a, hipStream_t st) {
  constexpr int smem = dq_smem_bytes<D, KS>();
  hipLaunchKernelGGL((attn_bwd_dq_kernel<D, C, DR, KS>), dim3((a.T / kBlockRows) * a.B * a.Hq), dim3(256 * KS),
                     smem, st, a);
}
// Causal D = 64 dQ: 2 key splits short, 3 from T = 1024 (A/B, profiles/attention_causal_d64_ks_r5.txt: T 2048
// 35.4 -> 32.4 us with 3; B4 T512 12.6 with 2 against 13.1)
constexpr int kDqCausalLongT = 1024;
template <int D, bool C, bool DR>
void launch_dq(const AttnArgs& a, hipStream_t st) {
  constexpr int KS = dq_ks<D, C>();
  if constexpr (D == 64 && C && DLTB_CAUSAL_KS_CAP && DLTB_DQ_KS64 > KS) {
    if (a.T >= kDqCausalLongT) return launch_dq_ks<D, C, DR, DLTB_DQ_KS64>(a, st);
  }
  launch_dq_ks<D, C, DR, KS>(a, st);
}
}  // namespace

// The dK/dV grid has one workgroup (4 waves, 1 wave / SIMD at D = 128) per key block and KV head.
// A causal grid is unbalanced (key block 0 sees every query tile, the last one a single tile) and
// when it is no deeper than the chip (Mistral-7B shape: 32 key blocks x 8 KV heads = 256) the
// step waits for the heaviest workgroup.  Splitting the G query heads of each KV group over
// several workgroups (fp32 partials + one reduce) makes the grid several waves deep, dispatched
// heaviest first.  DLTB_DKDV_GSPLIT = n forces n (1 = off).
int dltb_attn_dkdv_gsplit(int B, int T, int Hq, int Hkv, int causal) {
  const int G = Hq / Hkv;
  if (!causal || G < 2) return 1;
  static const int forced = [] {
    const char* e = getenv("DLTB_DKDV_GSPLIT");
    return e ? atoi(e) : 0;
  }();
  if (forced > 0) return G % forced == 0 ? forced : 1;
  const long wgs = (long)(T / kBlockRows) * B * Hkv;
  int s = 1;
  while (s < G && wgs * s < 2L * 256 && G % (2 * s) == 0) s *= 2;
  return s;
}

// part: 0 = dK/dV (key-major kernel), 1 = dQ (query-major kernel); both need delta
void dltb_attn_bwd_part(int part, const void* q, const void* k, const void* v, const void* dout,
                        const float* lse, const float* delta, const uint32_t* mask, void* out,
                        void* out2, long qs, long ks, long vs, long dos, long outs, long out2s,
                        int B, int T, int Hq, int Hkv, int D, float scale, int causal,
                        uint32_t thr16, float drop_scale, hipStream_t st, const void* o, long os,
                        int gsplit, float* part_buf) {
  AttnArgs a = make_args(q, k, v, qs, ks, vs, B, T, Hq, Hkv, scale, causal, thr16, drop_scale,
                         nullptr, 0);
  if (part == 0 && gsplit > 1 && part_buf && (Hq / Hkv) % gsplit == 0) {
    a.gsplit = gsplit;
    a.part = part_buf;
  }
  a.dout = (const bf16_t*)dout;
  a.do_stride = dos;
  a.lse = const_cast<float*>(lse);
  a.delta = delta;
  a.mask = mask;
  a.out = (bf16_t*)out;
  a.out_stride = outs;
  a.out2 = (bf16_t*)out2;
  a.out2_stride = out2s;
  a.o = part == 1 ? (const bf16_t*)o : nullptr;     // dQ pass computes and writes delta itself
  a.o_stride = os;
  if (part == 0)
    DLTB_ATTN_DISPATCH(launch_dkdv, D, causal != 0, thr16 != 0, a, st);
  else
    DLTB_ATTN_DISPATCH(launch_dq, D, causal != 0, thr16 != 0, a, st);
}
