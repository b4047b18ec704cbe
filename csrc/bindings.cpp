// pybind11 bindings of the dltb HIP kernels (module dltb._C).
//
// Thin adapters: validate devices/dtypes/shapes on the host (a wrong shape must never reach a
// kernel: an out-of-bounds access can reset every GPU of the node), pick the current HIP stream,
// and call the gfx950 launchers of launchers.h.  GEMMs stay in torch (hipBLASLt).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <cmath>

#include "launchers.h"

namespace {

using at::Tensor;
using c10::optional;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_cuda(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
}
void check_bf16(const Tensor& t, const char* name) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bf16");
}
void check_contig_bf16(const Tensor& t, const char* name) {
  check_bf16(t, name);
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}
void check_align16(const Tensor& t, const char* name) {
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name,
              " must be 16-byte aligned");
}

uint32_t thr_of(double p) {
  double t = p * 65536.0 + 0.5;
  if (t > 65536.0) t = 65536.0;
  return p > 0.0 ? (uint32_t)t : 0u;
}
float scale_of(double p) { return p > 0.0 ? (float)(1.0 / (1.0 - p)) : 1.f; }

const int64_t* seed_ptr(const optional<Tensor>& seed, double p) {
  if (p <= 0.0) return nullptr;
  TORCH_CHECK(seed.has_value(), "dropout p > 0 needs a seed tensor");
  check_cuda(*seed, "seed");
  TORCH_CHECK(seed->scalar_type() == at::kLong && seed->numel() >= 1, "seed must be int64[1]");
  return seed->data_ptr<int64_t>();
}

// caller-provided output (a view of a preallocated, layer-strided activation buffer) or a new tensor
Tensor out_or_new(const optional<Tensor>& out, const Tensor& like, const char* name) {
  if (!out.has_value()) return at::empty_like(like);
  check_contig_bf16(*out, name);
  TORCH_CHECK(out->sizes() == like.sizes(), name, ": output shape");
  check_align16(*out, name);
  return *out;
}

// ------------------------------------------------------------------------------------ norms
std::vector<Tensor> norm_fwd(const Tensor& x, const optional<Tensor>& r, const Tensor& w,
                             const optional<Tensor>& b, double eps, bool rms, double p,
                             const optional<Tensor>& seed, int64_t site, const optional<Tensor>& y_out) {
  check_contig_bf16(x, "x");
  check_contig_bf16(w, "w");
  const int64_t d = x.size(-1);
  const int64_t N = x.numel() / d;
  TORCH_CHECK(d % 8 == 0 && d <= 4096, "norm: d must be a multiple of 8 and <= 4096");
  TORCH_CHECK(w.numel() == d, "norm: weight size");
  if (!rms) {
    TORCH_CHECK(b.has_value(), "layernorm needs a bias");
    check_contig_bf16(*b, "b");
    TORCH_CHECK(b->numel() == d, "norm: bias size");
  }
  Tensor s;
  if (r.has_value()) {
    check_contig_bf16(*r, "r");
    TORCH_CHECK(r->sizes() == x.sizes(), "norm: residual shape");
    s = at::empty_like(x);
  }
  auto y = out_or_new(y_out, x, "norm_fwd y_out");
  auto fopt = x.options().dtype(at::kFloat);
  auto mean = rms ? Tensor() : at::empty({N}, fopt);
  auto rstd = at::empty({N}, fopt);
  dltb_norm_fwd(x.data_ptr(), r.has_value() ? r->data_ptr() : nullptr, w.data_ptr(),
                rms ? nullptr : b->data_ptr(), r.has_value() ? s.data_ptr() : nullptr,
                y.data_ptr(), rms ? nullptr : mean.data_ptr<float>(), rstd.data_ptr<float>(),
                (int)N, (int)d, (float)eps, rms, r.has_value() ? thr_of(p) : 0u, scale_of(p),
                r.has_value() ? seed_ptr(seed, p) : nullptr, site, cur_stream());
  return {s, y, mean, rstd};
}

Tensor norm_bwd(const Tensor& dy, const Tensor& s, const Tensor& w, const optional<Tensor>& mean,
                const Tensor& rstd, const optional<Tensor>& dres, const Tensor& gw,
                const optional<Tensor>& gb, bool accumulate, bool rms) {
  check_contig_bf16(dy, "dy");
  check_contig_bf16(s, "s");
  check_contig_bf16(w, "w");
  check_contig_bf16(gw, "gw");
  const int64_t d = dy.size(-1);
  const int64_t N = dy.numel() / d;
  TORCH_CHECK(s.sizes() == dy.sizes() && w.numel() == d && gw.numel() == d, "norm_bwd shapes");
  TORCH_CHECK(rstd.numel() == N, "norm_bwd: rstd size");
  if (!rms) {
    TORCH_CHECK(mean.has_value() && mean->numel() == N, "norm_bwd: mean");
    TORCH_CHECK(gb.has_value(), "layernorm bwd needs gb");
    check_contig_bf16(*gb, "gb");
    TORCH_CHECK(gb->numel() == d, "norm_bwd: gb size");
  }
  if (dres.has_value()) {
    check_contig_bf16(*dres, "dres");
    TORCH_CHECK(dres->sizes() == dy.sizes(), "norm_bwd: dres shape");
  }
  auto dx = at::empty_like(dy);
  const int P = dltb_norm_bwd_partials((int)N);
  auto part = at::empty({(int64_t)P * 2 * d}, dy.options().dtype(at::kFloat));
  dltb_norm_bwd(dy.data_ptr(), s.data_ptr(), w.data_ptr(),
                rms ? nullptr : mean->data_ptr<float>(), rstd.data_ptr<float>(),
                dres.has_value() ? dres->data_ptr() : nullptr, dx.data_ptr(),
                part.data_ptr<float>(), gw.data_ptr(), rms ? nullptr : gb->data_ptr(),
                accumulate ? 1 : 0, (int)N, (int)d, rms, cur_stream());
  return dx;
}

// ------------------------------------------------------------------------------ elementwise
Tensor gelu_fwd(const Tensor& f, const optional<Tensor>& out) {
  check_contig_bf16(f, "f");
  TORCH_CHECK(f.numel() % 8 == 0, "gelu: numel % 8");
  auto g = out_or_new(out, f, "gelu_fwd out");
  dltb_gelu_fwd(f.data_ptr(), g.data_ptr(), f.numel(), cur_stream());
  return g;
}

Tensor gelu_bwd(const Tensor& dg, const Tensor& f, const optional<Tensor>& db, bool accumulate) {
  check_contig_bf16(dg, "dg");
  check_contig_bf16(f, "f");
  TORCH_CHECK(dg.sizes() == f.sizes(), "gelu_bwd shapes");
  const int64_t k = f.size(-1);
  const int64_t N = f.numel() / k;
  TORCH_CHECK(k % 8 == 0, "gelu_bwd: k % 8");
  if (db.has_value()) {
    check_contig_bf16(*db, "db");
    TORCH_CHECK(db->numel() == k, "gelu_bwd: db size");
  }
  auto df = at::empty_like(dg);
  auto part = at::empty({(int64_t)dltb_colsum_partials((int)N) * k}, f.options().dtype(at::kFloat));
  dltb_gelu_bwd(dg.data_ptr(), f.data_ptr(), df.data_ptr(), part.data_ptr<float>(),
                db.has_value() ? db->data_ptr() : nullptr, accumulate ? 1 : 0, (int)N, (int)k,
                cur_stream());
  return df;
}

void colsum_into(const Tensor& src, const Tensor& out, bool accumulate) {
  check_contig_bf16(src, "src");
  check_contig_bf16(out, "out");
  const int64_t k = src.size(-1);
  const int64_t N = src.numel() / k;
  TORCH_CHECK(out.numel() == k && k % 8 == 0, "colsum shapes");
  auto part = at::empty({(int64_t)dltb_colsum_partials((int)N) * k}, src.options().dtype(at::kFloat));
  dltb_colsum(src.data_ptr(), part.data_ptr<float>(), out.data_ptr(), accumulate ? 1 : 0, (int)N,
              (int)k, cur_stream());
}

Tensor dropout(const optional<Tensor>& x, const Tensor& r, double p, const optional<Tensor>& seed,
               int64_t site) {
  check_contig_bf16(r, "r");
  const int64_t cols = r.size(-1);
  TORCH_CHECK(cols % 8 == 0, "dropout: last dim % 8");
  if (x.has_value()) {
    check_contig_bf16(*x, "x");
    TORCH_CHECK(x->sizes() == r.sizes(), "dropout_add shapes");
  }
  auto out = at::empty_like(r);
  dltb_dropout(x.has_value() ? x->data_ptr() : nullptr, r.data_ptr(), out.data_ptr(), r.numel(),
               (int)cols, thr_of(p), scale_of(p), seed_ptr(seed, p), site, cur_stream());
  return out;
}

Tensor swiglu_fwd(const Tensor& gu) {
  check_contig_bf16(gu, "gu");
  const int64_t F2 = gu.size(-1);
  TORCH_CHECK(F2 % 16 == 0, "swiglu: 2F % 16");
  const int64_t N = gu.numel() / F2;
  auto sizes = gu.sizes().vec();
  sizes.back() = F2 / 2;
  auto h = at::empty(sizes, gu.options());
  dltb_swiglu_fwd(gu.data_ptr(), h.data_ptr(), (int)N, (int)(F2 / 2), cur_stream());
  return h;
}

Tensor swiglu_bwd(const Tensor& dh, const Tensor& gu) {
  check_contig_bf16(dh, "dh");
  check_contig_bf16(gu, "gu");
  const int64_t F2 = gu.size(-1);
  const int64_t N = gu.numel() / F2;
  TORCH_CHECK(dh.numel() == N * F2 / 2, "swiglu_bwd shapes");
  auto dgu = at::empty_like(gu);
  dltb_swiglu_bwd(dh.data_ptr(), gu.data_ptr(), dgu.data_ptr(), (int)N, (int)(F2 / 2), cur_stream());
  return dgu;
}

void rope_(const Tensor& qkv, const Tensor& cosb, const Tensor& sinb, int64_t T, int64_t heads,
           int64_t D, bool inverse) {
  check_bf16(qkv, "qkv");
  TORCH_CHECK(qkv.dim() == 2 && qkv.stride(1) == 1, "rope: qkv must be a 2-D row-major view");
  check_cuda(cosb, "cos");
  TORCH_CHECK(cosb.scalar_type() == at::kFloat && sinb.scalar_type() == at::kFloat, "rope tables f32");
  TORCH_CHECK(cosb.is_contiguous() && sinb.is_contiguous(), "rope tables contiguous");
  TORCH_CHECK(D % 16 == 0, "rope: D % 16");
  TORCH_CHECK(cosb.numel() >= T * D / 2 && sinb.numel() >= T * D / 2, "rope table size");
  TORCH_CHECK(qkv.size(1) >= heads * D, "rope: heads * D exceeds row");
  const int64_t N = qkv.size(0);
  TORCH_CHECK(N % T == 0, "rope: rows % T");
  dltb_rope(qkv.data_ptr(), cosb.data_ptr<float>(), sinb.data_ptr<float>(), (int)N, (int)T,
            (int)heads, (int)D, (int)qkv.stride(0), inverse, cur_stream());
}

void f32_from_bf16_(const Tensor& dst, const Tensor& src, bool accumulate) {
  check_cuda(dst, "dst");
  check_contig_bf16(src, "src");
  TORCH_CHECK(dst.scalar_type() == at::kFloat && dst.is_contiguous(), "dst f32 contiguous");
  TORCH_CHECK(dst.numel() == src.numel() && src.numel() % 8 == 0, "cast sizes");
  check_align16(dst, "dst");
  check_align16(src, "src");
  dltb_f32_from_bf16(dst.data_ptr<float>(), src.data_ptr(), src.numel(), accumulate ? 1 : 0,
                     cur_stream());
}

// ------------------------------------------------------------------------------ embedding
Tensor embed_fwd(const Tensor& idx, const Tensor& wte, const Tensor& wpe, double p,
                 const optional<Tensor>& seed, int64_t site) {
  check_cuda(idx, "idx");
  TORCH_CHECK(idx.scalar_type() == at::kLong && idx.dim() == 2 && idx.is_contiguous(), "idx [B,T] int64");
  check_contig_bf16(wte, "wte");
  check_contig_bf16(wpe, "wpe");
  const int64_t B = idx.size(0), T = idx.size(1), d = wte.size(1);
  TORCH_CHECK(wpe.size(1) == d && wpe.size(0) >= T && d % 8 == 0, "embed shapes");
  auto x = at::empty({B, T, d}, wte.options());
  dltb_embed_fwd(idx.data_ptr<int64_t>(), wte.data_ptr(), wpe.data_ptr(), x.data_ptr(), (int)(B * T),
                 (int)T, (int)d, thr_of(p), scale_of(p), seed_ptr(seed, p), site, cur_stream());
  return x;
}

// dwte must already hold whatever it accumulates onto (zero it when nothing was written yet)
void embed_bwd(const Tensor& dx, const Tensor& idx, const optional<Tensor>& dwte,
               const optional<Tensor>& dwpe, bool accumulate_wpe, double p,
               const optional<Tensor>& seed, int64_t site) {
  check_contig_bf16(dx, "dx");
  TORCH_CHECK(idx.scalar_type() == at::kLong && idx.dim() == 2, "idx [B,T] int64");
  const int64_t B = idx.size(0), T = idx.size(1), d = dx.size(-1);
  TORCH_CHECK(dx.numel() == B * T * d, "embed_bwd: dx shape");
  const int64_t* sp = seed_ptr(seed, p);
  if (dwpe.has_value()) {
    check_contig_bf16(*dwpe, "dwpe");
    TORCH_CHECK(dwpe->size(1) == d && dwpe->size(0) >= T, "embed_bwd: dwpe shape");
    dltb_embed_bwd_pos(dx.data_ptr(), dwpe->data_ptr(), (int)B, (int)T, (int)dwpe->size(0), (int)d,
                       accumulate_wpe ? 1 : 0, thr_of(p), scale_of(p), sp, site, cur_stream());
  }
  if (dwte.has_value()) {
    check_contig_bf16(*dwte, "dwte");
    TORCH_CHECK(dwte->size(1) == d, "embed_bwd: dwte shape");
    auto flat = idx.reshape({-1}).contiguous();
    if (dltb_embed_bwd_tok_scan(dx.data_ptr(), flat.data_ptr<int64_t>(), dwte->data_ptr(), (int)(B * T),
                                (int)d, thr_of(p), scale_of(p), sp, site, cur_stream()))
      return;
    auto sorted = at::sort(flat);
    auto ids = std::get<0>(sorted).contiguous();
    auto perm = std::get<1>(sorted).contiguous();
    dltb_embed_bwd_tok(dx.data_ptr(), ids.data_ptr<int64_t>(), perm.data_ptr<int64_t>(),
                       dwte->data_ptr(), (int)(B * T), (int)d, thr_of(p), scale_of(p), sp, site,
                       cur_stream());
  }
}

// ------------------------------------------------------------------------------ xent
Tensor xent_fwd_bwd_(const Tensor& logits, const Tensor& targets, int64_t ignore_index) {
  check_contig_bf16(logits, "logits");
  check_cuda(targets, "targets");
  TORCH_CHECK(targets.scalar_type() == at::kLong && targets.is_contiguous(), "targets int64");
  const int64_t V = logits.size(-1);
  const int64_t N = logits.numel() / V;
  TORCH_CHECK(targets.numel() == N, "xent: targets size");
  TORCH_CHECK(V % 8 == 0 && V <= 131072, "xent: V % 8 and V <= 131072");
  auto loss = at::empty({N}, logits.options().dtype(at::kFloat));
  dltb_xent_fwd_bwd(logits.data_ptr(), targets.data_ptr<int64_t>(), loss.data_ptr<float>(), (int)N,
                    (int)V, ignore_index, cur_stream());
  return loss;
}

// mean loss over non-ignored targets, device side: returns f32[2] = (mean, max(count, 1))
Tensor xent_mean(const Tensor& loss_rows, const Tensor& targets, int64_t ignore_index) {
  check_cuda(loss_rows, "loss_rows");
  check_cuda(targets, "targets");
  TORCH_CHECK(loss_rows.scalar_type() == at::kFloat && loss_rows.is_contiguous(), "xent_mean: loss f32");
  TORCH_CHECK(targets.scalar_type() == at::kLong && targets.is_contiguous() &&
              targets.numel() == loss_rows.numel(), "xent_mean: targets int64 [N]");
  auto out = at::empty({2}, loss_rows.options());
  dltb_xent_mean(loss_rows.data_ptr<float>(), targets.data_ptr<int64_t>(), (int)loss_rows.numel(),
                 ignore_index, out.data_ptr<float>(), cur_stream());
  return out;
}

// y = x * num[0] / den[0] (device scalars); optionally stores the scale into g_out[0]
Tensor scale_by(const Tensor& x, const Tensor& num, const optional<Tensor>& den, const optional<Tensor>& g_out) {
  check_contig_bf16(x, "x");
  TORCH_CHECK(x.numel() % 8 == 0, "scale_by: numel % 8");
  check_cuda(num, "num");
  TORCH_CHECK(num.scalar_type() == at::kFloat && num.numel() >= 1, "scale_by: num f32");
  const float* dp = nullptr;
  if (den.has_value()) {
    check_cuda(*den, "den");
    TORCH_CHECK(den->scalar_type() == at::kFloat && den->numel() >= 1, "scale_by: den f32");
    dp = den->data_ptr<float>();
  }
  float* gp = nullptr;
  if (g_out.has_value()) {
    check_cuda(*g_out, "g_out");
    TORCH_CHECK(g_out->scalar_type() == at::kFloat && g_out->numel() >= 1, "scale_by: g_out f32");
    gp = g_out->data_ptr<float>();
  }
  auto y = at::empty_like(x);
  dltb_scale(x.data_ptr(), y.data_ptr(), x.numel(), num.data_ptr<float>(), dp, gp, cur_stream());
  return y;
}

// ------------------------------------------------------------------------------ optimizer
void adamw(const Tensor& master, const Tensor& exp_avg, const Tensor& exp_avg_sq,
           const Tensor& grad, const Tensor& blk_seg, const Tensor& blk_start,
           const Tensor& seg_ostart, const Tensor& seg_len, const Tensor& seg_dst,
           const optional<Tensor>& gscale, double lr, double beta1, double beta2, double eps,
           double wd, int64_t step, const optional<Tensor>& hp) {
  for (auto* t : {&master, &exp_avg, &exp_avg_sq}) {
    check_cuda(*t, "adam state");
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous(), "adam state f32 contiguous");
    check_align16(*t, "adam state");
  }
  check_cuda(grad, "grad");
  TORCH_CHECK(grad.is_contiguous(), "grad contiguous");
  TORCH_CHECK(master.numel() == exp_avg.numel() && master.numel() == exp_avg_sq.numel() &&
                  master.numel() == grad.numel(), "adam: state sizes differ");
  TORCH_CHECK(grad.scalar_type() == at::kFloat || grad.scalar_type() == at::kBFloat16, "grad dtype");
  TORCH_CHECK(blk_seg.scalar_type() == at::kInt && blk_start.scalar_type() == at::kLong, "adam tables");
  TORCH_CHECK(blk_seg.numel() == blk_start.numel(), "adam block tables");
  TORCH_CHECK(step >= 1, "adam: step >= 1");
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  const float* gs = nullptr;
  if (gscale.has_value()) {
    check_cuda(*gscale, "gscale");
    TORCH_CHECK(gscale->scalar_type() == at::kFloat, "gscale f32");
    gs = gscale->data_ptr<float>();
  }
  const float* hpp = nullptr;      // [lr, lr/bc1, 1/sqrt(bc2)] on the device: graph-replay safe
  if (hp.has_value()) {
    check_cuda(*hp, "hp");
    TORCH_CHECK(hp->scalar_type() == at::kFloat && hp->numel() >= 3, "adam hp: f32[>=3]");
    hpp = hp->data_ptr<float>();
  }
  dltb_adamw(master.data_ptr<float>(), exp_avg.data_ptr<float>(), exp_avg_sq.data_ptr<float>(),
             grad.data_ptr(), grad.scalar_type() == at::kBFloat16, blk_seg.data_ptr<int>(),
             blk_start.data_ptr<int64_t>(), (int)blk_seg.numel(), seg_ostart.data_ptr<int64_t>(),
             seg_len.data_ptr<int64_t>(), seg_dst.data_ptr<int64_t>(), gs, hpp, (float)lr, (float)beta1,
             (float)beta2, (float)eps, (float)wd, (float)(lr / bc1), (float)(1.0 / std::sqrt(bc2)),
             cur_stream());
}

void sumsq_(const Tensor& x, const Tensor& out) {
  check_cuda(x, "x");
  check_cuda(out, "out");
  TORCH_CHECK(x.is_contiguous() && x.numel() % 4 == 0, "sumsq: contiguous, numel % 4");
  TORCH_CHECK(out.scalar_type() == at::kFloat, "sumsq out f32");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "sumsq dtype");
  Tensor part = at::empty({dltb_sumsq_partials()}, out.options());
  dltb_sumsq(x.data_ptr(), x.scalar_type() == at::kBFloat16, x.numel(), out.data_ptr<float>(),
             part.data_ptr<float>(), cur_stream());
}

void clip_coef(const Tensor& norm_sq, double max_norm, const Tensor& coef,
               const optional<Tensor>& norm_out, double extra_scale) {
  check_cuda(norm_sq, "norm_sq");
  check_cuda(coef, "coef");
  dltb_clip_coef(norm_sq.data_ptr<float>(), (float)max_norm, coef.data_ptr<float>(),
                 norm_out.has_value() ? norm_out->data_ptr<float>() : nullptr, (float)extra_scale,
                 cur_stream());
}

// ------------------------------------------------------------------------------ attention
void check_attn_view(const Tensor& t, const char* name, int64_t rows, int64_t heads, int64_t D) {
  check_bf16(t, name);
  TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1, name, " must be a 2-D row-major view [B*T, >=H*D]");
  TORCH_CHECK(t.size(0) == rows && t.size(1) == heads * D, name, " shape mismatch");
  TORCH_CHECK(t.stride(0) % 8 == 0, name, " row stride must be a multiple of 8");
  check_align16(t, name);
}

void check_lse(const Tensor& t, int64_t n, const char* name) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == at::kFloat && t.numel() == n && t.is_contiguous(), name, " f32 [B,Hq,T]");
}

const uint32_t* mask_ptr(const optional<Tensor>& mask, uint32_t thr, int64_t B, int64_t T, int64_t Hq) {
  if (!thr) return nullptr;
  TORCH_CHECK(mask.has_value() && mask->is_cuda() && mask->scalar_type() == at::kInt &&
                  mask->numel() == dltb_attn_mask_words((int)B, (int)Hq, (int)T),
              "attention with dropout needs the packed mask of attn_mask()");
  return reinterpret_cast<const uint32_t*>(mask->data_ptr<int>());
}

int64_t attn_head_dim(const Tensor& q, int64_t B, int64_t T, int64_t Hq) {
  const int64_t D = q.size(1) / Hq;
  TORCH_CHECK(dltb_attn_supported((int)D, (int)T), "attention: needs D in {64,128} and T % 128 == 0");
  return D;
}

Tensor attn_mask(int64_t B, int64_t T, int64_t Hq, double p, const Tensor& seed, int64_t site,
                 const Tensor& like) {
  TORCH_CHECK(T % 128 == 0 && p > 0.0, "attn_mask: T % 128 and p > 0");
  auto mask = at::empty({dltb_attn_mask_words((int)B, (int)Hq, (int)T)}, like.options().dtype(at::kInt));
  dltb_attn_mask(reinterpret_cast<uint32_t*>(mask.data_ptr<int>()), (int)B, (int)T, (int)Hq, thr_of(p),
                 seed_ptr(seed, p), site, cur_stream());
  return mask;
}

std::vector<Tensor> attn_fwd(const Tensor& q, const Tensor& k, const Tensor& v,
                             const optional<Tensor>& mask, int64_t B, int64_t T, int64_t Hq,
                             int64_t Hkv, double scale, bool causal, double p,
                             const optional<Tensor>& o_out) {
  const int64_t D = attn_head_dim(q, B, T, Hq);
  TORCH_CHECK(Hq % Hkv == 0, "attention: Hq % Hkv");
  check_attn_view(q, "q", B * T, Hq, D);
  check_attn_view(k, "k", B * T, Hkv, D);
  check_attn_view(v, "v", B * T, Hkv, D);
  const uint32_t thr = thr_of(p);
  const uint32_t* mp = mask_ptr(mask, thr, B, T, Hq);
  dltb_attn_init_attributes();
  Tensor o;
  if (o_out.has_value()) {
    check_contig_bf16(*o_out, "attn_fwd o_out");
    TORCH_CHECK(o_out->dim() == 2 && o_out->size(0) == B * T && o_out->size(1) == Hq * D, "attn_fwd o_out shape");
    o = *o_out;
  } else {
    o = at::empty({B * T, Hq * D}, q.options());
  }
  auto lse = at::empty({B, Hq, T}, q.options().dtype(at::kFloat));
  dltb_attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr<float>(), mp,
                q.stride(0), k.stride(0), v.stride(0), o.stride(0), (int)B, (int)T, (int)Hq, (int)Hkv,
                (int)D, (float)scale, causal ? 1 : 0, thr, scale_of(p), cur_stream());
  return {o, lse};
}

Tensor attn_bwd_delta(const Tensor& o, const Tensor& dout, int64_t B, int64_t T, int64_t Hq) {
  const int64_t D = attn_head_dim(o, B, T, Hq);
  check_attn_view(o, "o", B * T, Hq, D);
  check_attn_view(dout, "dout", B * T, Hq, D);
  auto delta = at::empty({B, Hq, T}, o.options().dtype(at::kFloat));
  dltb_attn_bwd_delta(o.data_ptr(), dout.data_ptr(), delta.data_ptr<float>(), o.stride(0),
                      dout.stride(0), (int)B, (int)T, (int)Hq, (int)D, cur_stream());
  return delta;
}

// part 0: dK, dV (out = dk, out2 = dv); part 1: dQ (out = dq)
void attn_bwd_part(int64_t part, const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& dout,
                   const Tensor& lse, const Tensor& delta, const optional<Tensor>& mask,
                   const Tensor& out, const optional<Tensor>& out2, int64_t B, int64_t T, int64_t Hq,
                   int64_t Hkv, double scale, bool causal, double p, const optional<Tensor>& o) {
  const int64_t D = attn_head_dim(q, B, T, Hq);
  check_attn_view(q, "q", B * T, Hq, D);
  check_attn_view(k, "k", B * T, Hkv, D);
  check_attn_view(v, "v", B * T, Hkv, D);
  check_attn_view(dout, "dout", B * T, Hq, D);
  check_lse(lse, B * Hq * T, "lse");
  check_lse(delta, B * Hq * T, "delta");
  if (part == 0) {
    TORCH_CHECK(out2.has_value(), "dkdv needs dv");
    check_attn_view(out, "dk", B * T, Hkv, D);
    check_attn_view(*out2, "dv", B * T, Hkv, D);
  } else {
    check_attn_view(out, "dq", B * T, Hq, D);
  }
  if (o.has_value()) {            // dQ pass writes delta = rowsum(dO * O) for the dK/dV pass
    TORCH_CHECK(part == 1, "attn_bwd_part: o (fused delta) only for the dQ pass");
    check_attn_view(*o, "o", B * T, Hq, D);
  }
  const uint32_t thr = thr_of(p);
  const uint32_t* mp = mask_ptr(mask, thr, B, T, Hq);
  dltb_attn_init_attributes();
  int gsplit = 1;
  Tensor pbuf;
  if (part == 0) {
    gsplit = dltb_attn_dkdv_gsplit((int)B, (int)T, (int)Hq, (int)Hkv, causal ? 1 : 0);
    const bool vec_ok = reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0 &&
                        reinterpret_cast<uintptr_t>(out2->data_ptr()) % 16 == 0 &&
                        out.stride(0) % 8 == 0 && out2->stride(0) % 8 == 0;
    if (!vec_ok) gsplit = 1;
    if (gsplit > 1)
      pbuf = at::empty({gsplit * 2 * B * T * Hkv * D}, q.options().dtype(at::kFloat));
  }
  dltb_attn_bwd_part((int)part, q.data_ptr(), k.data_ptr(), v.data_ptr(), dout.data_ptr(),
                     lse.data_ptr<float>(), delta.data_ptr<float>(), mp, out.data_ptr(),
                     part == 0 ? out2->data_ptr() : nullptr, q.stride(0), k.stride(0), v.stride(0),
                     dout.stride(0), out.stride(0), part == 0 ? out2->stride(0) : 0, (int)B, (int)T,
                     (int)Hq, (int)Hkv, (int)D, (float)scale, causal ? 1 : 0, thr, scale_of(p),
                     cur_stream(), o.has_value() ? o->data_ptr() : nullptr, o.has_value() ? o->stride(0) : 0,
                     gsplit, gsplit > 1 ? pbuf.data_ptr<float>() : nullptr);
}

void attn_bwd(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& o, const Tensor& dout,
              const Tensor& lse, const optional<Tensor>& mask, const Tensor& dq, const Tensor& dk,
              const Tensor& dv, int64_t B, int64_t T, int64_t Hq, int64_t Hkv, double scale, bool causal,
              double p) {
  auto delta = attn_bwd_delta(o, dout, B, T, Hq);
  attn_bwd_part(0, q, k, v, dout, lse, delta, mask, dk, dv, B, T, Hq, Hkv, scale, causal, p, c10::nullopt);
  attn_bwd_part(1, q, k, v, dout, lse, delta, mask, dq, c10::nullopt, B, T, Hq, Hkv, scale, causal, p,
                c10::nullopt);
}

Tensor norm_bwd_dx(const Tensor& dy, const Tensor& s, const Tensor& w, const optional<Tensor>& mean,
                   const Tensor& rstd, const optional<Tensor>& dres, bool rms) {
  check_contig_bf16(dy, "dy");
  check_contig_bf16(s, "s");
  check_contig_bf16(w, "w");
  const int64_t d = dy.size(-1);
  const int64_t N = dy.numel() / d;
  TORCH_CHECK(d % 8 == 0 && d <= 4096 && s.sizes() == dy.sizes() && w.numel() == d, "norm_bwd_dx shapes");
  TORCH_CHECK(rstd.numel() == N && (rms || (mean.has_value() && mean->numel() == N)), "norm stats");
  if (dres.has_value()) {
    check_contig_bf16(*dres, "dres");
    TORCH_CHECK(dres->sizes() == dy.sizes(), "norm_bwd_dx: dres shape");
  }
  auto dx = at::empty_like(dy);
  dltb_norm_bwd_dx(dy.data_ptr(), s.data_ptr(), w.data_ptr(), rms ? nullptr : mean->data_ptr<float>(),
                   rstd.data_ptr<float>(), dres.has_value() ? dres->data_ptr() : nullptr, dx.data_ptr(),
                   (int)N, (int)d, rms, cur_stream());
  return dx;
}

// fused norm backward: (dx, part[K, P, d] f32) with K = (rms ? 1 : 2) + dx_sum; see norm.hip
std::tuple<Tensor, Tensor> norm_bwd_fused(const Tensor& dy, const Tensor& s, const Tensor& w,
                                          const optional<Tensor>& mean, const Tensor& rstd,
                                          const optional<Tensor>& dres, bool rms, bool dx_sum,
                                          const optional<Tensor>& dx_out, const optional<Tensor>& dm_out,
                                          double drop_p, const optional<Tensor>& seed, int64_t site) {
  check_contig_bf16(dy, "dy");
  check_contig_bf16(s, "s");
  check_contig_bf16(w, "w");
  const int64_t d = dy.size(-1);
  const int64_t N = dy.numel() / d;
  TORCH_CHECK(dltb_norm_bwd_fused_supported((int)d), "norm_bwd_fused: unsupported width");
  TORCH_CHECK(s.sizes() == dy.sizes() && w.numel() == d, "norm_bwd_fused shapes");
  TORCH_CHECK(rstd.numel() == N && (rms || (mean.has_value() && mean->numel() == N)), "norm stats");
  if (dres.has_value()) {
    check_contig_bf16(*dres, "dres");
    TORCH_CHECK(dres->sizes() == dy.sizes(), "norm_bwd_fused: dres shape");
  }
  auto dx = out_or_new(dx_out, dy, "norm_bwd_fused dx_out");
  void* dm = nullptr;
  if (dm_out.has_value()) {           // + the dropout backward of dx and ITS column sums (not dx's)
    TORCH_CHECK(!dx_sum, "norm_bwd_fused: dm_out and dx_sum are exclusive");
    check_contig_bf16(*dm_out, "dm_out");
    TORCH_CHECK(dm_out->sizes() == dy.sizes(), "norm_bwd_fused: dm_out shape");
    dm = dm_out->data_ptr();
  }
  const int64_t K = (rms ? 1 : 2) + ((dx_sum || dm) ? 1 : 0);
  auto part = at::empty({K, (int64_t)dltb_norm_bwd_fused_blocks((int)N), d}, dy.options().dtype(at::kFloat));
  dltb_norm_bwd_fused(dy.data_ptr(), s.data_ptr(), w.data_ptr(), rms ? nullptr : mean->data_ptr<float>(),
                      rstd.data_ptr<float>(), dres.has_value() ? dres->data_ptr() : nullptr, dx.data_ptr(),
                      part.data_ptr<float>(), (int)N, (int)d, rms, dx_sum, cur_stream(), dm,
                      dm ? thr_of(drop_p) : 0u, scale_of(drop_p), dm ? seed_ptr(seed, drop_p) : nullptr, site);
  return {dx, part};
}

void norm_bwd_dgamma(const Tensor& dy, const Tensor& s, const optional<Tensor>& mean, const Tensor& rstd,
                     const Tensor& gw, const optional<Tensor>& gb, bool accumulate, bool rms) {
  check_contig_bf16(dy, "dy");
  check_contig_bf16(s, "s");
  check_contig_bf16(gw, "gw");
  const int64_t d = dy.size(-1);
  const int64_t N = dy.numel() / d;
  TORCH_CHECK(s.sizes() == dy.sizes() && gw.numel() == d, "norm_bwd_dgamma shapes");
  TORCH_CHECK(rstd.numel() == N && (rms || (mean.has_value() && mean->numel() == N)), "norm stats");
  if (!rms) {
    TORCH_CHECK(gb.has_value(), "layernorm needs gb");
    check_contig_bf16(*gb, "gb");
    TORCH_CHECK(gb->numel() == d, "gb size");
  }
  const int P = dltb_norm_bwd_partials((int)N);
  auto part = at::empty({(int64_t)P * 2 * d}, dy.options().dtype(at::kFloat));
  dltb_norm_bwd_dgamma(dy.data_ptr(), s.data_ptr(), rms ? nullptr : mean->data_ptr<float>(),
                       rstd.data_ptr<float>(), part.data_ptr<float>(), gw.data_ptr(),
                       rms ? nullptr : gb->data_ptr(), accumulate ? 1 : 0, (int)N, (int)d, rms,
                       cur_stream());
}

// ------------------------------------------------------------------ batched column reductions
// colpart: one launch computing fp32 column partials of up to 3 segments (see colreduce.hip).
// Returns the partial tensors ([nout, P, k] f32; nout = 2 for LayerNorm segments).
std::vector<Tensor> colpart(const std::vector<int64_t>& kinds, const std::vector<Tensor>& a,
                            const std::vector<optional<Tensor>>& b,
                            const std::vector<optional<Tensor>>& dst,
                            const std::vector<optional<Tensor>>& mean,
                            const std::vector<optional<Tensor>>& rstd, double p,
                            const optional<Tensor>& seed, const std::vector<int64_t>& sites) {
  const size_t n = kinds.size();
  TORCH_CHECK(n >= 1 && n <= 3, "colpart: 1..3 segments");
  TORCH_CHECK(a.size() == n && b.size() == n && dst.size() == n && mean.size() == n && rstd.size() == n &&
              sites.size() == n, "colpart: list lengths");
  int64_t N0 = -1;
  std::vector<Tensor> parts;
  DltbColPartSeg segs[3];
  const int64_t* sp = nullptr;
  for (size_t i = 0; i < n; ++i) {
    const int kind = (int)kinds[i];
    check_contig_bf16(a[i], "colpart a");
    check_align16(a[i], "colpart a");
    const int64_t k = a[i].size(-1);
    const int64_t N = a[i].numel() / k;
    TORCH_CHECK(k % 8 == 0, "colpart: k % 8");
    if (N0 < 0) N0 = N;
    TORCH_CHECK(N == N0, "colpart: segments must share the row count");
    DltbColPartSeg& S = segs[i];
    S = DltbColPartSeg{};
    S.a = reinterpret_cast<const uint16_t*>(a[i].data_ptr());
    S.N = (int)N;
    S.k = (int)k;
    S.kind = kind;
    S.site = sites[i];
    if (kind == DLTB_COLPART_GELU || kind == DLTB_COLPART_LN || kind == DLTB_COLPART_RMS) {
      TORCH_CHECK(b[i].has_value(), "colpart: second input");
      check_contig_bf16(*b[i], "colpart b");
      TORCH_CHECK(b[i]->sizes() == a[i].sizes(), "colpart: b shape");
      S.b = reinterpret_cast<const uint16_t*>(b[i]->data_ptr());
    }
    if (kind == DLTB_COLPART_GELU || kind == DLTB_COLPART_DROP) {
      TORCH_CHECK(dst[i].has_value(), "colpart: dst");
      check_contig_bf16(*dst[i], "colpart dst");
      TORCH_CHECK(dst[i]->sizes() == a[i].sizes(), "colpart: dst shape");
      S.dst = reinterpret_cast<uint16_t*>(dst[i]->data_ptr());
    }
    if (kind == DLTB_COLPART_LN || kind == DLTB_COLPART_RMS) {
      TORCH_CHECK(rstd[i].has_value() && rstd[i]->numel() == N && rstd[i]->scalar_type() == at::kFloat,
                  "colpart: rstd");
      S.rstd = rstd[i]->data_ptr<float>();
      if (kind == DLTB_COLPART_LN) {
        TORCH_CHECK(mean[i].has_value() && mean[i]->numel() == N && mean[i]->scalar_type() == at::kFloat,
                    "colpart: mean");
        S.mean = mean[i]->data_ptr<float>();
      }
    }
    if (kind == DLTB_COLPART_DROP) sp = seed_ptr(seed, p);
    const int P = dltb_colpart_partials((int)N);
    Tensor part = at::empty({kind == DLTB_COLPART_LN ? 2 : 1, P, k}, a[i].options().dtype(at::kFloat));
    S.part = part.data_ptr<float>();
    parts.push_back(part);
  }
  dltb_colpart(segs, (int)n, dltb_colpart_partials((int)N0), thr_of(p), scale_of(p), sp, cur_stream());
  return parts;
}

// colreduce_multi: parts[i] ([P, k] f32, contiguous) summed into outs[i] (bf16, k elements)
void colreduce_multi(const std::vector<Tensor>& parts, const std::vector<Tensor>& outs,
                     const std::vector<bool>& accumulate) {
  const size_t n = parts.size();
  TORCH_CHECK(n >= 1 && n <= DLTB_COLRED_MAX && outs.size() == n && accumulate.size() == n,
              "colreduce_multi: 1..", DLTB_COLRED_MAX, " segments");
  DltbColRedSeg segs[DLTB_COLRED_MAX];
  for (size_t i = 0; i < n; ++i) {
    check_cuda(parts[i], "part");
    TORCH_CHECK(parts[i].scalar_type() == at::kFloat && parts[i].is_contiguous() && parts[i].dim() == 2,
                "colreduce_multi: part must be contiguous f32 [P, k]");
    check_contig_bf16(outs[i], "colreduce out");
    const int64_t k = parts[i].size(1);
    TORCH_CHECK(outs[i].numel() == k && k % 4 == 0, "colreduce_multi: out size / k % 4");
    check_align16(parts[i], "part");
    segs[i] = DltbColRedSeg{parts[i].data_ptr<float>(), reinterpret_cast<uint16_t*>(outs[i].data_ptr()),
                            (int)parts[i].size(0), (int)k, accumulate[i] ? 1 : 0};
  }
  dltb_colreduce_multi(segs, (int)n, cur_stream());
}

// dst[C, R] = src[R, C]^T (bf16, both contiguous)
void transpose_into(const Tensor& src, const Tensor& dst) {
  check_contig_bf16(src, "src");
  check_contig_bf16(dst, "dst");
  TORCH_CHECK(src.dim() == 2 && dst.dim() == 2 && dst.size(0) == src.size(1) && dst.size(1) == src.size(0),
              "transpose_into: shapes");
  TORCH_CHECK(src.size(1) % 4 == 0 && src.size(0) % 4 == 0, "transpose_into: dims % 4");
  dltb_transpose(src.data_ptr(), dst.data_ptr(), (int)src.size(0), (int)src.size(1), cur_stream());
}

// batched transpose: nb equally spaced [R, C] matrices starting at src (a 2-D view) -> [C, R] at
// dst; strides in elements.  The extents are checked against both storages.
void transpose_batched(const Tensor& src, const Tensor& dst, int64_t nb, int64_t sbs, int64_t dbs) {
  check_bf16(src, "src");
  check_bf16(dst, "dst");
  TORCH_CHECK(src.dim() == 2 && dst.dim() == 2 && src.is_contiguous() && dst.is_contiguous() &&
              dst.size(0) == src.size(1) && dst.size(1) == src.size(0), "transpose_batched: shapes");
  TORCH_CHECK(src.size(1) % 4 == 0 && src.size(0) % 4 == 0 && nb >= 1 && sbs >= 0 && dbs >= 0,
              "transpose_batched: dims % 4 / batch");
  TORCH_CHECK(nb == 1 || (sbs >= src.numel() && dbs >= dst.numel()), "transpose_batched: overlapping matrices");
  const int64_t es = 2;
  TORCH_CHECK((src.storage_offset() + (nb - 1) * sbs + src.numel()) * es <= (int64_t)src.storage().nbytes() &&
              (dst.storage_offset() + (nb - 1) * dbs + dst.numel()) * es <= (int64_t)dst.storage().nbytes(),
              "transpose_batched: batch exceeds the storage");
  dltb_transpose_batched(src.data_ptr(), dst.data_ptr(), (int)src.size(0), (int)src.size(1), (int)nb,
                         (long)sbs, (long)dbs, cur_stream());
}

// ------------------------------------------------------------------------------- GEMM
// layout "nt": a [M, K], b [N, K] -> out [M, N];  "tn": a [K, M], b [K, N] -> out [M, N]
// rows may be strided (views of fused buffers); the inner dimension must be contiguous.
bool gemm_supported(int64_t M, int64_t N, int64_t K, bool tn, int64_t cfg) {
  return dltb_gemm_supported((int)M, (int)N, (int)K, tn, (int)cfg);
}

Tensor gemm(const Tensor& a, const Tensor& b, const optional<Tensor>& out, const optional<Tensor>& bias,
            bool tn, bool accumulate, int64_t splits, int64_t cfg, int64_t pf, int64_t gm,
            const optional<Tensor>& alpha, int64_t stages) {
  check_bf16(a, "a");
  check_bf16(b, "b");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.stride(1) == 1 && b.stride(1) == 1, "gemm: 2-D, inner dim contiguous");
  const int64_t M = tn ? a.size(1) : a.size(0), K = tn ? a.size(0) : a.size(1);
  const int64_t N = tn ? b.size(1) : b.size(0);
  TORCH_CHECK((tn ? b.size(0) : b.size(1)) == K, "gemm: K mismatch");
  TORCH_CHECK(dltb_gemm_supported((int)M, (int)N, (int)K, tn, (int)cfg), "gemm: shape/tile not supported");
  TORCH_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0, "gemm: row strides must be 16-byte multiples");
  check_align16(a, "a");
  check_align16(b, "b");
  Tensor c;
  if (out.has_value()) {
    c = *out;
    check_bf16(c, "out");
    TORCH_CHECK(c.dim() == 2 && c.size(0) == M && c.size(1) == N && c.stride(1) == 1 && c.stride(0) % 4 == 0,
                "gemm: out shape / layout");
  } else {
    TORCH_CHECK(!accumulate, "gemm: accumulate needs out");
    c = at::empty({M, N}, a.options());
  }
  const void* bp = nullptr;
  if (bias.has_value()) {
    check_contig_bf16(*bias, "bias");
    TORCH_CHECK(bias->numel() == N, "gemm: bias size");
    bp = bias->data_ptr();
  }
  const float* ap = nullptr;
  if (alpha.has_value()) {
    check_cuda(*alpha, "alpha");
    TORCH_CHECK(alpha->scalar_type() == at::kFloat && alpha->numel() >= 1, "gemm: alpha f32 device scalar");
    ap = alpha->data_ptr<float>();
  }
  Tensor part;
  if (splits > 1) part = at::empty({splits, M, N}, a.options().dtype(at::kFloat));
  dltb_gemm(a.data_ptr(), b.data_ptr(), c.data_ptr(), bp, splits > 1 ? part.data_ptr<float>() : nullptr,
            a.stride(0), b.stride(0), c.stride(0), (int)M, (int)N, (int)K, tn, accumulate ? 1 : 0,
            (int)splits, (int)cfg, (int)pf, (int)gm, ap, cur_stream(), (int)stages);
  return c;
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "dltb gfx950 (MI355X) HIP kernels";
  m.def("norm_fwd", &norm_fwd, py::arg("x"), py::arg("r"), py::arg("w"), py::arg("b"), py::arg("eps"),
        py::arg("rms"), py::arg("p"), py::arg("seed"), py::arg("site"), py::arg("y_out") = py::none());
  m.def("norm_bwd", &norm_bwd);
  m.def("gelu_fwd", &gelu_fwd, py::arg("f"), py::arg("out") = py::none());
  m.def("gelu_bwd", &gelu_bwd);
  m.def("colsum_into", &colsum_into);
  m.def("dropout", &dropout);
  m.def("swiglu_fwd", &swiglu_fwd);
  m.def("swiglu_bwd", &swiglu_bwd);
  m.def("rope_", &rope_);
  m.def("f32_from_bf16_", &f32_from_bf16_);
  m.def("embed_fwd", &embed_fwd);
  m.def("embed_bwd", &embed_bwd);
  m.def("xent_fwd_bwd_", &xent_fwd_bwd_);
  m.def("adamw", &adamw);
  m.def("adamw_chunk", &dltb_adamw_chunk);
  m.def("sumsq_", &sumsq_);
  m.def("clip_coef", &clip_coef);
  m.def("attn_mask", &attn_mask);
  m.def("attn_fwd", &attn_fwd, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("mask"), py::arg("B"),
        py::arg("T"), py::arg("Hq"), py::arg("Hkv"), py::arg("scale"), py::arg("causal"), py::arg("p"),
        py::arg("o_out") = py::none());
  m.def("attn_bwd_delta", &attn_bwd_delta);
  m.def("attn_bwd_part", &attn_bwd_part, py::arg("part"), py::arg("q"), py::arg("k"), py::arg("v"),
        py::arg("dout"), py::arg("lse"), py::arg("delta"), py::arg("mask"), py::arg("out"), py::arg("out2"),
        py::arg("B"), py::arg("T"), py::arg("Hq"), py::arg("Hkv"), py::arg("scale"), py::arg("causal"),
        py::arg("p"), py::arg("o") = py::none());
  m.def("attn_bwd", &attn_bwd);
  m.def("norm_bwd_dx", &norm_bwd_dx);
  m.def("norm_bwd_dgamma", &norm_bwd_dgamma);
  m.def("norm_bwd_fused", &norm_bwd_fused, py::arg("dy"), py::arg("s"), py::arg("w"), py::arg("mean"),
        py::arg("rstd"), py::arg("dres"), py::arg("rms"), py::arg("dx_sum"), py::arg("dx_out") = py::none(),
        py::arg("dm_out") = py::none(), py::arg("drop_p") = 0.0, py::arg("seed") = py::none(),
        py::arg("site") = 0);
  m.def("norm_bwd_fused_supported", [](int64_t d) { return dltb_norm_bwd_fused_supported((int)d); });
  m.def("colpart", &colpart);
  m.def("gemm", &gemm, py::arg("a"), py::arg("b"), py::arg("out"), py::arg("bias"), py::arg("tn"),
        py::arg("accumulate"), py::arg("splits") = 1, py::arg("cfg") = 0, py::arg("pf") = 0, py::arg("gm") = 1,
        py::arg("alpha") = py::none(), py::arg("stages") = 0);
  m.def("gemm_supported", &gemm_supported);
  m.def("xent_mean", &xent_mean);
  m.def("scale_by", &scale_by, py::arg("x"), py::arg("num"), py::arg("den") = py::none(),
        py::arg("g_out") = py::none());
  m.def("transpose_into", &transpose_into);
  m.def("transpose_batched", &transpose_batched);
  m.def("colreduce_multi", &colreduce_multi);
  m.def("arch", []() { return std::string("gfx950"); });
}
