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
// Dropout uses the counter hash of common.h (row = (b*Hq + h)*T + q, col = key).  The keep-mask is
// generated ONCE per call by a full-occupancy kernel as packed bits laid out for the forward's lane
// mapping: word (bh, t, h, q) holds, in bit 16n + i, the decision for key 64t + 32n + (i&3) +
// 8(i>>2) + 4h of query q — so forward and dQ lanes read one coalesced word per 64-key tile and the
// dK/dV kernel stages 4 words per query row in LDS.  The hash runs 1x instead of 3x, and the
// softmax kernels pay 2 VALU ops per probability for dropout.
#include "common.h"

namespace {

typedef __bf16 bfx8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

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
};

DLTB_DEV f32x16 mfma32(bfx8 a, bfx8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

template <int D>
DLTB_DEV int swz(int row) {
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

// accumulator registers 8s .. 8s+7 -> bf16 B operand of k-step s
DLTB_DEV bfx8 acc_to_frag(const f32x16& x, int s) {
  bfx8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (__bf16)x[8 * s + j];
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
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      uint2 o;
      o.x = pack_bf2(acc[dt][4 * g + 0] * scale, acc[dt][4 * g + 1] * scale);
      o.y = pack_bf2(acc[dt][4 * g + 2] * scale, acc[dt][4 * g + 3] * scale);
      *reinterpret_cast<uint2*>(dst_row + dt * 32 + 8 * g + 4 * h) = o;
    }
  }
}

// =============================================================================== dropout mask
// word (bh, t, h, q) at ((bh*nT + t)*2 + h)*T + q; bit 16n + i <-> key 64t + 32n + (i&3) + 8(i>>2) + 4h
__global__ __launch_bounds__(256) void attn_mask_kernel(uint32_t* __restrict__ mask, long BH, int T,
                                                        uint32_t thr16, const int64_t* __restrict__ seed_ptr,
                                                        int64_t site) {
  const int nT = T / kTile;
  const long total = BH * nT * 2 * T;
  const uint64_t seed = site_seed(seed_ptr, site);
  for (long wi = blockIdx.x * 256L + threadIdx.x; wi < total; wi += (long)gridDim.x * 256) {
    const int q = (int)(wi % T);
    long rest = wi / T;
    const int h = (int)(rest & 1);
    rest >>= 1;
    const int t = (int)(rest % nT);
    const long bh = rest / nT;
    const uint32_t rk = rng_row_key(seed, (uint32_t)(bh * T + q));
    uint32_t bits = 0;
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        const uint32_t key = (uint32_t)(t * kTile + 32 * n + (i & 3) + 8 * (i >> 2) + 4 * h);
        const uint32_t hsh = rng_pair(rk, rng_col_key(seed, key));
        bits |= (keep_lo(hsh, thr16) ? 1u : 0u) << (16 * n + i);
        bits |= (keep_hi(hsh, thr16) ? 1u : 0u) << (16 * n + i + 1);
      }
    mask[wi] = bits;
  }
}

// =============================================================================== forward
template <int D, bool CAUSAL, bool DROP>
__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnArgs P) {
  constexpr int TB = kTile * D * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, h = lane >> 5;
  const int bh = blockIdx.y, b = bh / P.Hq, hq = bh % P.Hq, hk = hq / (P.Hq / P.Hkv);
  const int T = P.T;
  const int nT = T / kTile;
  const int q0 = blockIdx.x * kBlockRows + w * 32;
  const int qi = q0 + r;

  bfx8 qf[D / 16];
  {
    const bf16_t* qrow = P.q + ((long)b * T + qi) * P.q_stride + hq * D;
#pragma unroll
    for (int s = 0; s < D / 16; ++s) qf[s] = __builtin_bit_cast(bfx8, ld16<uint4>(qrow + 16 * s + 8 * h));
  }
  int nt = nT;
  if (CAUSAL) nt = min(nt, (blockIdx.x * kBlockRows + kBlockRows - 1) / kTile + 1);
  const bf16_t* kbase = P.k + (long)b * T * P.k_stride + hk * D;
  const bf16_t* vbase = P.v + (long)b * T * P.v_stride + hk * D;
  const uint32_t* mrow = DROP ? P.mask + ((long)bh * nT * 2 + h) * T + qi : nullptr;
  const float c = P.scale * kLog2e;

  TileLoader<D> lk, lv;
  lk.load(kbase, P.k_stride, 0, tid);
  lv.load(vbase, P.v_stride, 0, tid);
  uint32_t mw_next = DROP ? mrow[0] : 0u;
  lk.store(smem, tid);
  lv.store(smem + TB, tid);
  __syncthreads();

  f32x16 oacc[D / 32];
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt) oacc[dt] = f32x16{};
  float m = -INFINITY, l = 0.f;   // m in scaled log2 units

  for (int t = 0; t < nt; ++t) {
    const char* kt = smem + (t & 1) * 2 * TB;
    const char* vt = kt + TB;
    const uint32_t mw = mw_next;
    if (t + 1 < nt) {
      lk.load(kbase, P.k_stride, (t + 1) * kTile, tid);
      lv.load(vbase, P.v_stride, (t + 1) * kTile, tid);
      if (DROP) mw_next = mrow[(long)(t + 1) * 2 * T];
    }
    const int kv0 = t * kTile;
    if (!CAUSAL || kv0 <= q0 + 31) {
      f32x16 sacc[2];
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        sacc[n] = f32x16{};
#pragma unroll
        for (int s = 0; s < D / 16; ++s) sacc[n] = mfma32(row_frag<D>(kt, 32 * n + r, 2 * s + h), qf[s], sacc[n]);
      }
      float mx = -INFINITY;
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float v = sacc[n][i];
          if (CAUSAL) {
            const int key = kv0 + 32 * n + (i & 3) + 8 * (i >> 2) + 4 * h;
            if (key > qi) v = -INFINITY;
            sacc[n][i] = v;
          }
          mx = fmaxf(mx, v);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mnew = fmaxf(m, mx * c);
      const float alpha = __builtin_amdgcn_exp2f(m - mnew);
      m = mnew;
      float ls = 0.f;
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float p = __builtin_amdgcn_exp2f(fmaf(sacc[n][i], c, -mnew));
          ls += p;
          sacc[n][i] = (!DROP || ((mw >> (16 * n + i)) & 1u)) ? p : 0.f;
        }
      l = l * alpha + ls;
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt) oacc[dt] *= alpha;
#pragma unroll
      for (int n = 0; n < 2; ++n) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bfx8 pf = acc_to_frag(sacc[n], s2);
#pragma unroll
          for (int dt = 0; dt < D / 32; ++dt)
            oacc[dt] = mfma32(tr_frag<D>(vt, 32 * n + 16 * s2, dt * 32, lane), pf, oacc[dt]);
        }
      }
    }
    if (t + 1 < nt) {
      char* nk = smem + ((t + 1) & 1) * 2 * TB;
      lk.store(nk, tid);
      lv.store(nk + TB, tid);
    }
    __syncthreads();
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
template <int D>
constexpr int dkdv_smem_bytes() {
  return 2 * (2 * kTile * D * 2 + 2 * kTile * 4 + kTile * 16);
}

template <int D, bool CAUSAL, bool DROP>
__global__ __launch_bounds__(256) void attn_bwd_dkdv_kernel(AttnArgs P) {
  constexpr int TB = kTile * D * 2;
  constexpr int SB = dkdv_smem_bytes<D>() / 2;   // Q tile, dO tile, lse2[64], delta[64], mask[64][4]
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, h = lane >> 5;
  const int bk = blockIdx.y, b = bk / P.Hkv, hk = bk % P.Hkv;
  const int G = P.Hq / P.Hkv;
  const int T = P.T;
  const int nT = T / kTile;
  const int kblk0 = blockIdx.x * kBlockRows;
  const int k0 = kblk0 + w * 32;
  const int key = k0 + r;
  // this lane's bit in the packed mask words (see attn_mask_kernel)
  const int hbit = (r >> 2) & 1;
  const int jbit = 16 * (w & 1) + ((r & 3) | (((r >> 3) & 3) << 2));
  const int msub = (w >> 1) * 2 + hbit;

  bfx8 kf[D / 16], vf[D / 16];
  {
    const bf16_t* krow = P.k + ((long)b * T + key) * P.k_stride + hk * D;
    const bf16_t* vrow = P.v + ((long)b * T + key) * P.v_stride + hk * D;
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      kf[s] = __builtin_bit_cast(bfx8, ld16<uint4>(krow + 16 * s + 8 * h));
      vf[s] = __builtin_bit_cast(bfx8, ld16<uint4>(vrow + 16 * s + 8 * h));
    }
  }
  f32x16 dk[D / 32], dv[D / 32];
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt) { dk[dt] = f32x16{}; dv[dt] = f32x16{}; }

  const float c = P.scale * kLog2e;
  const int t_begin = CAUSAL ? kblk0 / kTile : 0;

  for (int g = 0; g < G; ++g) {
    const int hq = hk * G + g;
    const long bq = (long)b * P.Hq + hq;
    const bf16_t* qbase = P.q + (long)b * T * P.q_stride + hq * D;
    const bf16_t* dobase = P.dout + (long)b * T * P.do_stride + hq * D;
    TileLoader<D> lq, ldo;
    float vl = 0.f, vd = 0.f;
    uint32_t mword = 0;
    auto load_small = [&](int t) {
      if (tid < kTile) {
        vl = P.lse[bq * T + t * kTile + tid] * kLog2e;
        vd = P.delta[bq * T + t * kTile + tid];
      }
      if (DROP) {
        const int row = tid >> 2, sb = tid & 3;
        mword = P.mask[((bq * nT + (blockIdx.x * 2 + (sb >> 1))) * 2 + (sb & 1)) * T + t * kTile + row];
      }
    };
    auto store_small = [&](char* base) {
      float* f = reinterpret_cast<float*>(base + 2 * TB);
      if (tid < kTile) {
        f[tid] = vl;
        f[kTile + tid] = vd;
      }
      if (DROP) reinterpret_cast<uint32_t*>(f + 2 * kTile)[tid] = mword;
    };
    lq.load(qbase, P.q_stride, t_begin * kTile, tid);
    ldo.load(dobase, P.do_stride, t_begin * kTile, tid);
    load_small(t_begin);
    lq.store(smem, tid);
    ldo.store(smem + TB, tid);
    store_small(smem);
    __syncthreads();
    for (int t = t_begin; t < nT; ++t) {
      const int bufi = (t - t_begin) & 1;
      const char* qt = smem + bufi * SB;
      const char* dt_ = qt + TB;
      const float* lse2 = reinterpret_cast<const float*>(qt + 2 * TB);
      const float* dlt = lse2 + kTile;
      const uint32_t* mws = reinterpret_cast<const uint32_t*>(dlt + kTile);
      if (t + 1 < nT) {
        lq.load(qbase, P.q_stride, (t + 1) * kTile, tid);
        ldo.load(dobase, P.do_stride, (t + 1) * kTile, tid);
        load_small(t + 1);
      }
#pragma unroll
      for (int mm = 0; mm < 2; ++mm) {
        const int qb = t * kTile + 32 * mm;
        if (CAUSAL && qb + 31 < k0) continue;   // every query < every key of this wave
        f32x16 sa = f32x16{}, dp = f32x16{};
#pragma unroll
        for (int s = 0; s < D / 16; ++s) {
          sa = mfma32(row_frag<D>(qt, 32 * mm + r, 2 * s + h), kf[s], sa);
          dp = mfma32(row_frag<D>(dt_, 32 * mm + r, 2 * s + h), vf[s], dp);
        }
        f32x16 pd, ds;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int ql = 32 * mm + 8 * g4 + 4 * h;   // rows ql .. ql+3 for regs 4*g4 .. 4*g4+3
          const float4 L = *reinterpret_cast<const float4*>(lse2 + ql);
          const float4 Dl = *reinterpret_cast<const float4*>(dlt + ql);
          const float Lv[4] = {L.x, L.y, L.z, L.w};
          const float Dv[4] = {Dl.x, Dl.y, Dl.z, Dl.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int i = 4 * g4 + e;
            float p = __builtin_amdgcn_exp2f(fmaf(sa[i], c, -Lv[e]));
            if (CAUSAL && key > qb + 8 * g4 + 4 * h + e) p = 0.f;
            if (DROP) {
              const bool keep = (mws[(ql + e) * 4 + msub] >> jbit) & 1u;
              pd[i] = keep ? p : 0.f;
              ds[i] = p * ((keep ? dp[i] * P.drop_scale : 0.f) - Dv[e]);
            } else {
              pd[i] = p;
              ds[i] = p * (dp[i] - Dv[e]);
            }
          }
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bfx8 pf = acc_to_frag(pd, s2);
          const bfx8 sf = acc_to_frag(ds, s2);
#pragma unroll
          for (int d_ = 0; d_ < D / 32; ++d_) {
            dv[d_] = mfma32(tr_frag<D>(dt_, 32 * mm + 16 * s2, d_ * 32, lane), pf, dv[d_]);
            dk[d_] = mfma32(tr_frag<D>(qt, 32 * mm + 16 * s2, d_ * 32, lane), sf, dk[d_]);
          }
        }
      }
      if (t + 1 < nT) {
        char* nb = smem + ((t + 1 - t_begin) & 1) * SB;
        lq.store(nb, tid);
        ldo.store(nb + TB, tid);
        store_small(nb);
      }
      __syncthreads();
    }
  }
  bf16_t* dkrow = P.out + ((long)b * T + key) * P.out_stride + hk * D;
  bf16_t* dvrow = P.out2 + ((long)b * T + key) * P.out2_stride + hk * D;
  store_acc_rows<D>(dkrow, dk, P.scale, h);
  store_acc_rows<D>(dvrow, dv, DROP ? P.drop_scale : 1.f, h);
}

// =============================================================================== dQ
template <int D, bool CAUSAL, bool DROP>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(AttnArgs P) {
  constexpr int TB = kTile * D * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, h = lane >> 5;
  const int bh = blockIdx.y, b = bh / P.Hq, hq = bh % P.Hq, hk = hq / (P.Hq / P.Hkv);
  const int T = P.T;
  const int nT = T / kTile;
  const int q0 = blockIdx.x * kBlockRows + w * 32;
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
  const float lse2 = P.lse[bq * T + qi] * kLog2e;
  const float dl = P.delta[bq * T + qi];
  const uint32_t* mrow = DROP ? P.mask + ((long)bq * nT * 2 + h) * T + qi : nullptr;
  const float c = P.scale * kLog2e;
  int nt = nT;
  if (CAUSAL) nt = min(nt, (blockIdx.x * kBlockRows + kBlockRows - 1) / kTile + 1);
  const bf16_t* kbase = P.k + (long)b * T * P.k_stride + hk * D;
  const bf16_t* vbase = P.v + (long)b * T * P.v_stride + hk * D;

  TileLoader<D> lk, lv;
  lk.load(kbase, P.k_stride, 0, tid);
  lv.load(vbase, P.v_stride, 0, tid);
  uint32_t mw_next = DROP ? mrow[0] : 0u;
  lk.store(smem, tid);
  lv.store(smem + TB, tid);
  __syncthreads();

  f32x16 dq[D / 32];
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt) dq[dt] = f32x16{};

  for (int t = 0; t < nt; ++t) {
    const char* kt = smem + (t & 1) * 2 * TB;
    const char* vt = kt + TB;
    const uint32_t mw = mw_next;
    if (t + 1 < nt) {
      lk.load(kbase, P.k_stride, (t + 1) * kTile, tid);
      lv.load(vbase, P.v_stride, (t + 1) * kTile, tid);
      if (DROP) mw_next = mrow[(long)(t + 1) * 2 * T];
    }
    const int kv0 = t * kTile;
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      if (CAUSAL && kv0 + 32 * n > q0 + 31) continue;
      f32x16 sa = f32x16{}, dp = f32x16{};
#pragma unroll
      for (int s = 0; s < D / 16; ++s) {
        sa = mfma32(row_frag<D>(kt, 32 * n + r, 2 * s + h), qf[s], sa);
        dp = mfma32(row_frag<D>(vt, 32 * n + r, 2 * s + h), of[s], dp);
      }
      f32x16 ds;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float p = __builtin_amdgcn_exp2f(fmaf(sa[i], c, -lse2));
        if (CAUSAL && kv0 + 32 * n + (i & 3) + 8 * (i >> 2) + 4 * h > qi) p = 0.f;
        float dpv = dp[i];
        if (DROP) dpv = ((mw >> (16 * n + i)) & 1u) ? dpv * P.drop_scale : 0.f;
        ds[i] = p * (dpv - dl);
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bfx8 sf = acc_to_frag(ds, s2);
#pragma unroll
        for (int dt = 0; dt < D / 32; ++dt)
          dq[dt] = mfma32(tr_frag<D>(kt, 32 * n + 16 * s2, dt * 32, lane), sf, dq[dt]);
      }
    }
    if (t + 1 < nt) {
      char* nk = smem + ((t + 1) & 1) * 2 * TB;
      lk.store(nk, tid);
      lv.store(nk + TB, tid);
    }
    __syncthreads();
  }
  bf16_t* dqrow = P.out + ((long)b * T + qi) * P.out_stride + hq * D;
  store_acc_rows<D>(dqrow, dq, P.scale, h);
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
  return a;
}

}  // namespace

bool dltb_attn_supported(int D, int T) { return (D == 64 || D == 128) && T % kBlockRows == 0; }

long dltb_attn_mask_words(int B, int Hq, int T) { return (long)B * Hq * (T / kTile) * 2 * T; }

namespace {

template <int D, bool C, bool DR>
void set_attrs() {
  (void)hipFuncSetAttribute((const void*)attn_fwd_kernel<D, C, DR>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 4 * kTile * D * 2);
  (void)hipFuncSetAttribute((const void*)attn_bwd_dq_kernel<D, C, DR>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 4 * kTile * D * 2);
  (void)hipFuncSetAttribute((const void*)attn_bwd_dkdv_kernel<D, C, DR>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, dkdv_smem_bytes<D>());
}

template <int D, bool C, bool DR>
void launch_fwd(const AttnArgs& a, hipStream_t st) {
  dim3 grid(a.T / kBlockRows, a.B * a.Hq);
  hipLaunchKernelGGL((attn_fwd_kernel<D, C, DR>), grid, dim3(256), 4 * kTile * D * 2, st, a);
}

template <int D, bool C, bool DR>
void launch_bwd(const AttnArgs& a, const AttnArgs& kv, hipStream_t st) {
  dim3 gkv(a.T / kBlockRows, a.B * a.Hkv);
  hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, C, DR>), gkv, dim3(256), dkdv_smem_bytes<D>(), st, kv);
  dim3 gq(a.T / kBlockRows, a.B * a.Hq);
  hipLaunchKernelGGL((attn_bwd_dq_kernel<D, C, DR>), gq, dim3(256), 4 * kTile * D * 2, st, a);
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
  const long words = dltb_attn_mask_words(B, Hq, T);
  long g = (words + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(attn_mask_kernel, dim3(g), dim3(256), 0, st, mask, (long)B * Hq, T, thr16, seed, site);
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
  dim3 gkv(a.T / kBlockRows, a.B * a.Hkv);
  hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, C, DR>), gkv, dim3(256), dkdv_smem_bytes<D>(), st, a);
}
template <int D, bool C, bool DR>
void launch_dq(const AttnArgs& a, hipStream_t st) {
  dim3 gq(a.T / kBlockRows, a.B * a.Hq);
  hipLaunchKernelGGL((attn_bwd_dq_kernel<D, C, DR>), gq, dim3(256), 4 * kTile * D * 2, st, a);
}
}  // namespace

// part: 0 = dK/dV (key-major kernel), 1 = dQ (query-major kernel); both need delta
void dltb_attn_bwd_part(int part, const void* q, const void* k, const void* v, const void* dout,
                        const float* lse, const float* delta, const uint32_t* mask, void* out,
                        void* out2, long qs, long ks, long vs, long dos, long outs, long out2s,
                        int B, int T, int Hq, int Hkv, int D, float scale, int causal,
                        uint32_t thr16, float drop_scale, hipStream_t st) {
  AttnArgs a = make_args(q, k, v, qs, ks, vs, B, T, Hq, Hkv, scale, causal, thr16, drop_scale,
                         nullptr, 0);
  a.dout = (const bf16_t*)dout;
  a.do_stride = dos;
  a.lse = const_cast<float*>(lse);
  a.delta = delta;
  a.mask = mask;
  a.out = (bf16_t*)out;
  a.out_stride = outs;
  a.out2 = (bf16_t*)out2;
  a.out2_stride = out2s;
  if (part == 0)
    DLTB_ATTN_DISPATCH(launch_dkdv, D, causal != 0, thr16 != 0, a, st);
  else
    DLTB_ATTN_DISPATCH(launch_dq, D, causal != 0, thr16 != 0, a, st);
}
