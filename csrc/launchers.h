// Host launch entry points of the dltb HIP kernels (implemented in csrc/*.hip, compiled by hipcc
// for gfx950 without torch headers; bindings.cpp adapts them to at::Tensor).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

// norm.hip
void dltb_norm_fwd(const void* x, const void* r, const void* w, const void* b, void* s_out,
                   void* y, float* mean, float* rstd, int N, int d, float eps, bool rms,
                   uint32_t thr16, float drop_scale, const int64_t* seed, int64_t site,
                   hipStream_t st);
// norm_fwd + the attention-dropout mask of (B, T, Hq) in one launch (horizontal fusion)
void dltb_norm_fwd_mask(const void* x, const void* r, const void* w, const void* b, void* s_out, void* y,
                        float* mean, float* rstd, int N, int d, float eps, bool rms, uint32_t thr16,
                        float drop_scale, const int64_t* seed, int64_t site, uint32_t* mask, int B, int T,
                        int Hq, uint32_t mask_thr16, const int64_t* mask_seed, int64_t mask_site, hipStream_t st,
                        int g_begin = 0, int g_end = -1);   // tile groups [g_begin, g_end) of the mask
int dltb_norm_bwd_partials(int N);
void dltb_norm_bwd_dx(const void* dy, const void* s, const void* w, const float* mean,
                      const float* rstd, const void* dres, void* dx, int N, int d, bool rms,
                      hipStream_t st);
void dltb_norm_bwd_dgamma(const void* dy, const void* s, const float* mean, const float* rstd,
                          float* part, void* gw, void* gb, int accumulate, int N, int d, bool rms,
                          hipStream_t st);
void dltb_norm_bwd(const void* dy, const void* s, const void* w, const float* mean,
                   const float* rstd, const void* dres, void* dx, float* part, void* gw, void* gb,
                   int accumulate, int N, int d, bool rms, hipStream_t st);
// fused dx + column partials; part: [(rms ? 1 : 2) + dxsum][blocks(N)][d] fp32
bool dltb_norm_bwd_fused_supported(int d);
int dltb_norm_bwd_fused_blocks(int N);
// dm != nullptr: also dm = dropout_bwd(dx) (site / thr16 / drop_scale / seed) and its column sums
bool dltb_norm_bwd_fused(const void* dy, const void* s, const void* w, const float* mean,
                         const float* rstd, const void* dres, void* dx, float* part, int N, int d,
                         bool rms, bool dxsum, hipStream_t st, void* dm = nullptr, uint32_t thr16 = 0,
                         float drop_scale = 1.f, const int64_t* seed = nullptr, int64_t site = 0);

// elementwise.hip
void dltb_gelu_fwd(const void* f, void* g, long n, hipStream_t st);
void dltb_gelu_fwd_grad(const void* f, void* g, void* gp, long n, hipStream_t st);   // g = GELU(f), gp = GELU'(f)
int dltb_colsum_partials(int N);
void dltb_gelu_bwd(const void* dg, const void* f, void* df, float* part, void* db, int accumulate,
                   int N, int k, hipStream_t st);
void dltb_colsum(const void* src, float* part, void* out, int accumulate, int N, int k,
                 hipStream_t st);
void dltb_dropout(const void* x, const void* r, void* out, long n, int cols, uint32_t thr16,
                  float scale, const int64_t* seed, int64_t site, hipStream_t st);
void dltb_swiglu_fwd(const void* gu, void* h, int N, int F, hipStream_t st);
void dltb_swiglu_bwd(const void* dh, const void* gu, void* dgu, int N, int F, hipStream_t st);
void dltb_rope(void* qkv, const float* cosb, const float* sinb, int N, int T, int heads, int D,
               int stride, bool inverse, hipStream_t st);
void dltb_f32_from_bf16(float* dst, const void* src, long n, int accumulate, hipStream_t st);
void dltb_transpose(const void* src, void* dst, int R, int C, hipStream_t st);
// nb matrices [R, C] at element stride sbs (src) / dbs (dst) -> [C, R] each, one launch
void dltb_transpose_batched(const void* src, void* dst, int R, int C, int nb, long sbs, long dbs,
                            hipStream_t st);

// comm_emu.hip: one emulated RCCL collective (DLTB_COMM=emulate:N) -- `channels` paced workgroups
// that read `traffic` (`passes` times) and write dst[r * rep_stride + j] = scale * src[j]
void dltb_comm_emu(const void* traffic, long traffic_bytes, int passes, void* dst, const void* src, long n,
                   int elem, float scale, int replicas, long rep_stride, float alpha_us, float beta_us,
                   int channels, hipStream_t st);

// embedding.hip
void dltb_embed_fwd(const int64_t* idx, const void* wte, const void* wpe, void* x, int N, int T,
                    int d, uint32_t thr16, float scale, const int64_t* seed, int64_t site,
                    hipStream_t st);
void dltb_embed_bwd_pos(const void* dx, void* dwpe, int B, int T, int P, int d, int accumulate,
                        uint32_t thr16, float scale, const int64_t* seed, int64_t site,
                        hipStream_t st);
bool dltb_embed_bwd_tok_scan(const void* dx, const int64_t* ids, void* dwte, int N, int d, long V,
                             uint32_t thr16, float scale, const int64_t* seed, int64_t site,
                             hipStream_t st);
void dltb_embed_bwd_tok(const void* dx, const int64_t* sorted_ids, const int64_t* perm,
                        void* dwte, int N, int d, long V, uint32_t thr16, float scale,
                        const int64_t* seed, int64_t site, hipStream_t st);

// xent.hip
void dltb_xent_fwd_bwd(void* logits, const int64_t* targets, float* loss, int N, int V,
                       int64_t ignore_index, hipStream_t st);

// adamw.hip
int dltb_adamw_chunk();
void dltb_adamw(float* master, float* exp_avg, float* exp_avg_sq, const void* grad, bool grad_bf16,
                const int* blk_seg, const int64_t* blk_start, int nblocks, const int64_t* seg_ostart,
                const int64_t* seg_len, const int64_t* seg_dst, const float* gscale, const float* hp,
                float lr, float beta1, float beta2, float eps, float wd, float step_size,
                float inv_sqrt_bc2, int grid_cap, hipStream_t st);   // grid_cap 0: one block per row
int dltb_sumsq_partials();
void dltb_sumsq(const void* x, bool bf16, long n, float* out, float* part, hipStream_t st);
void dltb_clip_coef(const float* norm_sq, float max_norm, float* coef, float* norm_out,
                    float extra_scale, hipStream_t st);
void dltb_fill_f32(float* x, long n, float v, hipStream_t st);
// dynamic loss scaling step (adamw.hip): state f32[4] = [scale, tracker, steps taken, skipped]
void dltb_amp_step(const float* norm_sq, float* state, float* coef, float* norm_out, float* hp,
                   float max_norm, float extra_scale, float beta1, float beta2, float growth,
                   float backoff, int growth_interval, hipStream_t st);

// attention.hip
bool dltb_attn_supported(int D, int T);
long dltb_attn_mask_words(int B, int Hq, int T);
void dltb_attn_mask(uint32_t* mask, int B, int T, int Hq, uint32_t thr16, const int64_t* seed,
                    int64_t site, hipStream_t st);
void dltb_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse,
                   const uint32_t* mask, long qs, long ks, long vs, long os, int B, int T, int Hq,
                   int Hkv, int D, float scale, int causal, uint32_t thr16, float drop_scale,
                   hipStream_t st);
void dltb_attn_bwd_delta(const void* o, const void* dout, float* delta, long os, long dos, int B,
                         int T, int Hq, int D, hipStream_t st);
void dltb_attn_bwd_part(int part, const void* q, const void* k, const void* v, const void* dout,
                        const float* lse, const float* delta, const uint32_t* mask, void* out,
                        void* out2, long qs, long ks, long vs, long dos, long outs, long out2s,
                        int B, int T, int Hq, int Hkv, int D, float scale, int causal,
                        uint32_t thr16, float drop_scale, hipStream_t st, const void* o = nullptr,
                        long os = 0, int gsplit = 1, float* part_buf = nullptr);
// dK/dV workgroups per KV head for a causal GQA backward (1 = one workgroup sums the whole group)
int dltb_attn_dkdv_gsplit(int B, int T, int Hq, int Hkv, int causal);
void dltb_attn_init_attributes();

// ---- batched column reductions (colreduce.hip)
#ifndef DLTB_LAUNCHER_TYPES   // types once (launchers_f16.h repeats only the declarations)
#define DLTB_LAUNCHER_TYPES
enum { DLTB_COLPART_PLAIN = 0, DLTB_COLPART_GELU = 1, DLTB_COLPART_DROP = 2, DLTB_COLPART_LN = 3,
       DLTB_COLPART_RMS = 4 };
#define DLTB_COLRED_MAX 64   // segments per colreduce_multi launch (kernel-argument struct: 2 KiB)
struct DltbColPartSeg {
  const uint16_t* a;
  const uint16_t* b;
  uint16_t* dst;
  const float* mean;
  const float* rstd;
  float* part;
  int N, k, kind;
  int64_t site;
};
struct DltbColRedSeg {
  const float* part;
  uint16_t* out;
  int P, k, accumulate;
};
#endif
int dltb_colpart_partials(int N);
void dltb_colpart(const DltbColPartSeg* segs, int nseg, int P, uint32_t thr16, float drop_scale,
                  const int64_t* seed, hipStream_t st);
void dltb_colreduce_multi(const DltbColRedSeg* segs, int nseg, hipStream_t st);

// ---- gemm.hip: C[M,N] = A B (+bias) (+C); NT: A [M][K], B [N][K]; TN: A [K][M], B [K][N]
bool dltb_gemm_supported(int M, int N, int K, bool tn, int cfg);
int dltb_gemm(const void* a, const void* b, void* c, const void* bias, float* part, long lda, long ldb,
              long ldc, int M, int N, int K, bool tn, int accumulate, int splits, int cfg, int pf, int gm,
              const float* alpha, hipStream_t st, int stages = 0);

// ---- gemm_tn.hip: C[b][M][N] (+)= A[b][K][M]^T B[b][K][N] (weight gradients dY^T X), bf16, 256 x 256 tiles,
// M, N multiples of 256, K of 64 (>= 128)
bool dltb_gemm_tn_supported(int M, int N, int K);
int dltb_gemm_tn(const void* a, const void* b, void* c, long lda, long ldb, long ldc, long sa, long sb, long sc,
                 int M, int N, int K, int batch, int accumulate, hipStream_t st);

// ---- gemm_rs.hip: C[M,N] = A[M][K] B[N][K]^T (+bias) (+C), bf16, register-staged operands (the step's per-layer kernel)
int dltb_gemm_rs_pick(int M, int N, int K);
bool dltb_gemm_rs_supported(int M, int N, int K, int cfg);
int dltb_gemm_rs(const void* a, const void* b, void* c, const void* bias, long lda, long ldb, long ldc, int M,
                 int N, int K, int accumulate, int cfg, int gm, hipStream_t st, const void* aux = nullptr,
                 float* part = nullptr, void* gout = nullptr);
// C = A B^T + bias and gout = GELU(C) (of the rounded C) from one launch (fp32-image kernels)
bool dltb_gemm_rs_gelu_supported(int M, int N, int K, int cfg);
int dltb_gemm_rs_bm(int cfg);
// C = (A B^T) * aux (elementwise, rounded once) with per-m-tile fp32 column partials of C (the dGELU epilogue)
bool dltb_gemm_rs_aux_supported(int M, int N, int K, int cfg);

// device-scalar helpers (head backward: no host sync)
void dltb_xent_mean(const float* loss, const int64_t* targets, int N, int64_t ignore_index, float* out,
                    hipStream_t st);
void dltb_scale(const void* x, void* y, long n, const float* num, const float* den, float* g_out,
                hipStream_t st);

