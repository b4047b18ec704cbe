"""TinyGPT — the reference benchmark model, re-built as fused per-unit autograd Functions.

Reference: ``benchmarking/train_harness.py:36-131`` (TinyGPT + TransformerBlock).  Parameter names,
shapes, tying and initialisation match the reference exactly so state dicts are interchangeable:

    transformer.wte.weight [V, d]  (tied with lm_head.weight)     transformer.wpe.weight [block, d]
    transformer.h.{i}.ln_1.{weight,bias}   .attn.in_proj_{weight [3d, d], bias [3d]}
    transformer.h.{i}.attn.out_proj.{weight, bias}   .ln_2.{weight,bias}
    transformer.h.{i}.mlp.0.{weight [4d, d], bias}   .mlp.2.{weight [d, 4d], bias}
    transformer.ln_f.{weight,bias}

Semantics reproduced from the reference: NON-causal attention (no mask), dropout
p on the embedding sum, the attention probabilities and the MLP output, pre-LN blocks, exact-erf
GELU, learned absolute positions, tied head, ``cross_entropy(ignore_index=-1)``.  Dead work of the
reference is not performed: ``ln_1`` is evaluated once (it is called 3x on the same input at
``train_harness.py:127``) and the head-averaged attention weights (``need_weights=True``) are never
computed.  The fused head returns ``logits=None`` when a loss is requested (the logits buffer is
overwritten by the softmax-xent gradient in place); pass ``return_logits=True`` to get them.

Per block (N = B*T tokens):  h1 = LN1(x); qkv = h1 Win^T + b; o = FlashAttn(qkv); a = o Wo^T + b;
x1 = x + a; h2 = LN2(x1) (one fused kernel); f = h2 W1^T + b; g = GELU(f); m = g W2^T + b;
x2 = x1 + dropout(m).  GEMMs are hipBLASLt (torch), everything else is dltb._C on the GPU.
"""
import math
from types import SimpleNamespace

import torch
import torch.nn as nn

from ..ops import functional as F_
from ..parallel.runtime import EAGER, Unit
from .config import ModelConfig

LN_EPS = 1e-5


class _MHAParams(nn.Module):
    """Parameter container with nn.MultiheadAttention's names (in_proj_weight, out_proj.*)."""

    def __init__(self, d):
        super().__init__()
        self.in_proj_weight = nn.Parameter(torch.empty(3 * d, d))
        self.in_proj_bias = nn.Parameter(torch.zeros(3 * d))
        self.out_proj = nn.Linear(d, d)
        nn.init.xavier_uniform_(self.in_proj_weight)    # nn.MultiheadAttention._reset_parameters
        nn.init.zeros_(self.out_proj.bias)


class TinyGPTBlock(nn.Module):
    def __init__(self, d, n_head, dropout):
        super().__init__()
        self.ln_1 = nn.LayerNorm(d)
        self.attn = _MHAParams(d)
        self.ln_2 = nn.LayerNorm(d)
        self.mlp = nn.Sequential(nn.Linear(d, 4 * d), nn.GELU(), nn.Linear(4 * d, d), nn.Dropout(dropout))

    def param_list(self):
        return [("ln_1.weight", self.ln_1.weight), ("ln_1.bias", self.ln_1.bias),
                ("attn.in_proj_weight", self.attn.in_proj_weight), ("attn.in_proj_bias", self.attn.in_proj_bias),
                ("attn.out_proj.weight", self.attn.out_proj.weight), ("attn.out_proj.bias", self.attn.out_proj.bias),
                ("ln_2.weight", self.ln_2.weight), ("ln_2.bias", self.ln_2.bias),
                ("mlp.0.weight", self.mlp[0].weight), ("mlp.0.bias", self.mlp[0].bias),
                ("mlp.2.weight", self.mlp[2].weight), ("mlp.2.bias", self.mlp[2].bias)]


# ============================================================================ fused Functions
# Measured and removed (round 2 toggle pruning; records under profiles/ab_*.jsonl): dropout mask /
# weight gradients / dQ on side streams (slower: two under-filling kernels slow each other down),
# a standalone residual+dropout kernel (the fused LayerNorm form is faster), and the consumer's
# LayerNorm backward forming the producer's MLP Dropout backward (neutral).


class _EmbedFn(torch.autograd.Function):
    """Token + position embedding.  The tied token table is a parameter of the HEAD unit (whose
    backward runs first and writes its dense gradient), so engines reduce it right after the
    head, under all block backwards; this unit owns only the position table.  The token rows of
    this backward are handed to ``rt.embedding_backward``: added to the head's dense part in place,
    or -- where the table's collective already ran -- exchanged sparsely (parallel/replicated.py,
    parallel/sharded.py)."""

    @staticmethod
    def forward(ctx, anchor, idx, model):
        rt, unit = model.rt, model.unit_embed
        (tu, ti), (_, pi) = model.tok_slot, model.pos_slot
        own = rt.acquire(unit)
        wpe = own[pi]
        wte = own[ti] if tu is unit else rt.acquire_tied(tu)[ti]
        p = model.drop_p
        x = F_.embed_fwd(idx, wte, wpe, p, rt.seed, model.site_embed)
        rt.release_forward(unit)
        ctx.model, ctx.idx = model, idx
        return x.view(-1, x.shape[-1])

    @staticmethod
    def backward(ctx, dx):
        model = ctx.model
        rt, unit = model.rt, model.unit_embed
        rt.acquire_backward(unit)
        rt.embedding_backward(model.tok_slot, model.pos_slot, dx.contiguous(), ctx.idx, model.drop_p, rt.seed,
                              model.site_embed)
        rt.grads_ready(unit)
        rt.release_backward(unit)
        return None, None, None


class _BlockFn(torch.autograd.Function):
    """One transformer block.  Inputs (x_in, m_in) / outputs (x1, m): a block hands the NEXT
    consumer its residual x1 and its un-dropped MLP output m, and the consumer's first LayerNorm
    forms x2 = x1 + Dropout(m) in the same kernel (norm_fwd with a residual; x2 is stored as that
    LayerNorm's residual stream), so the MLP dropout costs no launch of its own.  Gradient
    convention between the fused Functions: the consumer returns d(x2) for x1 and None for m; the
    producing block applies Dropout's backward itself (fused with the fc2 bias column sum)."""

    @staticmethod
    def forward(ctx, x_in, m_in, model, i):
        ctx.set_materialize_grads(False)
        rt, unit = model.rt, model.unit_blocks[i]
        (ln1w, ln1b, win, bin_, wo, bo, ln2w, ln2b, w1, b1, w2, b2) = rt.acquire(unit)
        B, T = model._cur_bt
        cfg = model.cfg
        H, d = cfg.n_head, cfg.n_embd
        p = model.drop_p
        lb = model.layer_buffer(i)          # layer-strided GEMM operands (batched weight gradients)
        # LN1 (with the previous block's MLP dropout + residual) and this block's attention-dropout
        # mask: one launch on the GPU.  With mask_split the previous block's LN2 launch already
        # generated the first half of this mask (model._next_amask) and LN1 adds the second half.
        prev, model._next_amask = model._next_amask, None
        x, h1, mean1, rstd1, amask = F_.norm_fwd_mask(
            x_in, m_in, ln1w, ln1b, LN_EPS, False, p if m_in is not None else 0.0, rt.seed,
            model.site_mlp(i - 1) if m_in is not None else 0, lb and lb.h1, B, T, H, p, model.site_attn(i),
            mask_out=prev, part=1 if prev is not None else None)
        if m_in is None:                    # block 0: the embedding output is the residual stream
            x = x_in
        qkv = F_.linear_fwd(h1, win, bin_)
        o, lse, amask = F_.attn_fwd(qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:], B, T, H, H,
                                    1.0 / math.sqrt(d // H), False, p, rt.seed, model.site_attn(i),
                                    amask, o_out=lb and lb.o)
        a = F_.linear_fwd(o, wo, bo)
        if model.mask_split and p > 0 and i + 1 < cfg.n_layer and x.is_cuda:
            # LN2 (latency-bound) beside the first half of the NEXT block's attention-dropout mask
            x1, h2, mean2, rstd2, model._next_amask = F_.norm_fwd_mask(
                x, a, ln2w, ln2b, LN_EPS, False, 0.0, rt.seed, 0, lb and lb.h2, B, T, H, p,
                model.site_attn(i + 1), part=0)
        else:
            x1, h2, mean2, rstd2 = F_.norm_fwd(x, a, ln2w, ln2b, LN_EPS, False, y_out=lb and lb.h2)
        # fc1 + GELU in one own-GEMM launch when the table has a GELU-epilogue row (bias = 3)
        fg = F_.linear_fwd_gelu(h2, w1, b1, g_out=lb and lb.g)
        if fg is not None:
            f, g = fg
            dgelu = False
        else:
            f = F_.linear_fwd(h2, w1, b1)
            # dGELU-epilogue path (own-GEMM table): keep GELU'(f) for the backward instead of f
            dgelu = f.is_cuda and F_.dgelu_fused(f.shape[0], f.shape[1], w2.shape[0], f.dtype)
            if dgelu:
                g, f = F_.gelu_fwd_grad(f, out=lb and lb.g)
            else:
                g = F_.gelu_fwd(f, out=lb and lb.g)
        m = F_.linear_fwd(g, w2, b2)        # Dropout(m) + x1 happens in the consumer's LayerNorm
        rt.release_forward(unit)
        ctx.model, ctx.i, ctx.lb = model, i, lb
        ctx.dgelu = dgelu                   # saved f is GELU'(f): the backward takes the dGELU-epilogue GEMM
        ctx.fused_prev = m_in is not None   # LN1 applied the previous block's MLP dropout
        ctx.saved = (x, h1, mean1, rstd1, qkv, o, lse, amask, x1, h2, mean2, rstd2, f, g)
        return x1, m

    @staticmethod
    def backward(ctx, dx2, dm_in):
        # dx2 = d(x1 + Dropout(m)) from the consumer.  m's gradient (Dropout backward, with the fc2
        # bias column sum) comes from the consumer block's LN1 backward kernel (dm_in, engines whose
        # gradient slots may be written ahead) or is formed here
        model, i = ctx.model, ctx.i
        rt, unit = model.rt, model.unit_blocks[i]
        (x, h1, mean1, rstd1, qkv, o, lse, amask, x1, h2, mean2, rstd2, f, g) = ctx.saved
        ctx.saved = None
        (ln1w, ln1b, win, bin_, wo, bo, ln2w, ln2b, w1, b1, w2, b2) = rt.acquire_backward(unit)
        B, T = model._cur_bt
        cfg = model.cfg
        H, d = cfg.n_head, cfg.n_embd
        p = model.drop_p
        dx2 = dx2.contiguous()
        s = [rt.grad_slot(unit, j) for j in range(12)]
        lb = ctx.lb

        def wgrad(j, dy, xin, names):      # dW_j (+)= dy^T xin: now, or queued and batched by the engine
            if lb is not None and lb.window:    # window-wide: once, at the last micro-step, all tokens
                if lb.full is not None:
                    rt.wgrad(unit, j, getattr(lb.full, names[0]), getattr(lb.full, names[1]), s[j][0], False)
                return
            rt.wgrad(unit, j, dy, xin, s[j][0], s[j][1])

        # the 8 bias / LayerNorm column sums: fused partials, reduced by ONE launch per block (or,
        # with the engine's shared reducer at world size 1, one launch for all blocks)
        shared = rt.grad_reducer()
        red = shared if shared is not None else F_.GradReducer()
        # MLP
        if dm_in is not None:
            dm = dm_in
        else:
            dm = F_.dropout_bwd_bias(dx2, p, rt.seed, model.site_mlp(i), s[11][0], s[11][1], red,
                                     out=lb and lb.dm)
        wgrad(10, dm, g, ("dm", "g"))
        w2t = rt.weight_t(unit, 10, w2)
        df = None
        if ctx.dgelu:                   # f holds GELU'(f): dGELU and the fc1 bias partials in the GEMM epilogue
            df = F_.dgelu_backward(dm, w2, w2t, f, s[9][0], s[9][1], red, out=lb and lb.df)
        else:
            dg = F_.linear_dgrad(dm, w2, w2t)
            df = F_.gelu_bwd(dg, f, s[9][0], s[9][1], red, out=lb and lb.df)
        wgrad(8, df, h2, ("df", "h2"))
        w1t = rt.weight_t(unit, 8, w1)
        dh2 = F_.linear_dgrad(df, w1, w1t)
        dx1 = F_.norm_bwd(dh2, x1, ln2w, mean2, rstd2, dx2, s[6][0], s[7][0], s[6][1], False,
                          red, bias=("dx", s[5][0], s[5][1]), dx_out=lb and lb.dx1)
        # attention
        wgrad(4, dx1, o, ("dx1", "o"))
        do = F_.linear_dgrad(dx1, wo, rt.weight_t(unit, 4, wo))
        dqkv = torch.empty_like(qkv) if lb is None else lb.dqkv
        F_.attn_bwd(qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:], o, do, lse, amask,
                    dqkv[:, :d], dqkv[:, d:2 * d], dqkv[:, 2 * d:], B, T, H, H,
                    1.0 / math.sqrt(d // H), False, p, rt.seed, model.site_attn(i))
        wgrad(2, dqkv, h1, ("dqkv", "h1"))
        wint = rt.weight_t(unit, 2, win)
        dh1 = F_.linear_dgrad(dqkv, win, wint)
        drop_prev = None
        if ctx.fused_prev and rt.grad_write_ahead and dx2.is_cuda:
            # the previous block's Dropout(m') backward and fc2 bias partials, formed with dx by the
            # LN1 backward kernel (one colpart launch less per layer: -0.6 % per micro-step,
            # profiles/fused_dropout_bwd_ab_r6.txt)
            ps = rt.grad_slot(model.unit_blocks[i - 1], 11)
            plb = model.layer_buffer(i - 1) if lb is not None else None
            drop_prev = (p, rt.seed, model.site_mlp(i - 1), plb and plb.dm, ps[0], ps[1])
        dx = F_.norm_bwd(dh1, x, ln1w, mean1, rstd1, dx1, s[0][0], s[1][0], s[0][1], False,
                         red, bias=(dqkv, s[3][0], s[3][1]), drop=drop_prev)
        dm_prev = None
        if drop_prev is not None:
            dx, dm_prev = dx
        if shared is None:
            red.flush()
        rt.grads_ready(unit)
        rt.release_backward(unit)
        return dx, dm_prev, None, None


class _HeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x_in, m_in, model, targets, return_logits):
        rt = model.rt
        tu, ti = model.tok_slot
        hp = rt.acquire(model.unit_head)
        lnw, lnb = hp[0], hp[1]
        wte = hp[ti] if tu is model.unit_head else rt.acquire_tied(tu)[ti]
        if m_in is None:
            x = x_in
            _, h, mean, rstd = F_.norm_fwd(x, None, lnw, lnb, LN_EPS, False)
        else:                               # last block's x1 + Dropout(m), fused into ln_f
            x, h, mean, rstd = F_.norm_fwd(x_in, m_in, lnw, lnb, LN_EPS, False, model.drop_p, rt.seed,
                                           model.site_mlp(len(model.unit_blocks) - 1))
        logits = F_.linear_fwd(h, wte)
        if targets is None:
            rt.release_forward(model.unit_head)
            ctx.mark_non_differentiable(logits)
            ctx.no_loss = True
            return logits, logits.new_zeros(())
        kept = logits.clone() if return_logits else None
        tg = targets.reshape(-1)
        loss_rows = F_.xent_fwd_bwd_(logits, tg, -1)
        lc = F_.xent_mean(loss_rows, tg, -1)          # (mean, count) on the device
        loss, count = lc[0], lc[1:2]
        rt.release_forward(model.unit_head)
        ctx.model, ctx.no_loss = model, False
        ctx.saved = (x, h, mean, rstd, logits, count)
        out_logits = kept if kept is not None else logits.new_empty(0)
        ctx.mark_non_differentiable(out_logits)
        return out_logits, loss

    @staticmethod
    def backward(ctx, dlogits_unused, dloss):
        if ctx.no_loss:
            return None, None, None, None, None
        model = ctx.model
        rt = model.rt
        (x, h, mean, rstd, dl, count) = ctx.saved
        ctx.saved = None
        tu, ti = model.tok_slot
        hp = rt.acquire_backward(model.unit_head)
        lnw, lnb = hp[0], hp[1]
        wte = hp[ti] if tu is model.unit_head else rt.acquire_tied(tu)[ti]
        dw, acc_w = rt.grad_slot(tu, ti)                          # tied lm_head / wte (dense part)
        hs, g = F_.scale_by(h, dloss, count)                      # g = dloss / count (device)
        F_.linear_wgrad(dl, hs, dw, None, acc_w)
        dh = F_.head_dgrad(dl, wte, rt.weight_t(tu, ti, wte), g)
        gw, acc = rt.grad_slot(model.unit_head, 0)
        gb, _ = rt.grad_slot(model.unit_head, 1)
        dx = F_.norm_bwd(dh, x, lnw, mean, rstd, None, gw, gb, acc, False)
        rt.grads_ready(model.unit_head)
        rt.release_backward(model.unit_head)
        return dx, None, None, None, None


# ============================================================================ module
class TinyGPT(nn.Module):
    """Reference-compatible TinyGPT (train_harness.py:36-105) on fused MI355X kernels."""

    def __init__(self, cfg: ModelConfig):
        super().__init__()
        self.cfg = cfg
        d = cfg.n_embd
        self.transformer = nn.ModuleDict({
            "wte": nn.Embedding(cfg.vocab_size, d),
            "wpe": nn.Embedding(cfg.block_size, d),
            "drop": nn.Dropout(cfg.dropout),
            "h": nn.ModuleList([TinyGPTBlock(d, cfg.n_head, cfg.dropout) for _ in range(cfg.n_layer)]),
            "ln_f": nn.LayerNorm(d),
        })
        self.lm_head = nn.Linear(d, cfg.vocab_size, bias=False)
        self.transformer["wte"].weight = self.lm_head.weight       # weight tying (train_harness.py:61)
        self.apply(self._init_weights)
        self.rt = EAGER
        self.drop_p = cfg.dropout
        self._lbufs = None
        self._lbuf_key = None
        # each attention-dropout mask is generated in two halves, beside the previous block's LN2
        # and beside this block's LN1 (both latency-bound row norms that leave VALU issue idle)
        self.mask_split = True         # (attribute, not an env switch: tests compare both paths)
        self._next_amask = None
        self._build_units()

    @staticmethod
    def _init_weights(module):
        if isinstance(module, nn.Linear):
            nn.init.normal_(module.weight, mean=0.0, std=0.02)
            if module.bias is not None:
                nn.init.zeros_(module.bias)
        elif isinstance(module, nn.Embedding):
            nn.init.normal_(module.weight, mean=0.0, std=0.02)
        elif isinstance(module, nn.LayerNorm):
            nn.init.zeros_(module.bias)
            nn.init.ones_(module.weight)

    def _build_units(self):
        t = self.transformer
        # the tied token table (wte = lm_head.weight) is the head unit's third parameter: the head's
        # backward, the first of the step, completes its dense gradient (see _EmbedFn), so engines reduce
        # it right after the head instead of after the last backward op (round 3: emulated DDP N = 8
        # exposed comm 2.01 -> 1.27 ms, profiles/emulated_ab_tail_tie_r3.txt)
        wpe = [("transformer.wpe.weight", t["wpe"].weight)]
        wte = [("transformer.wte.weight", t["wte"].weight)]
        self.unit_embed = Unit("embed", wpe, 0)
        self.unit_blocks = [Unit(f"h.{i}", [(f"transformer.h.{i}.{n}", p) for n, p in blk.param_list()], i + 1)
                            for i, blk in enumerate(t["h"])]
        self.unit_head = Unit("head", [("transformer.ln_f.weight", t["ln_f"].weight),
                                       ("transformer.ln_f.bias", t["ln_f"].bias)] + wte,
                              len(self.unit_blocks) + 1)
        self.tok_slot = (self.unit_head, 2)
        self.pos_slot = (self.unit_embed, 0)

    def units(self):
        """Units in forward order (the engines reverse it for backward-ordered buckets)."""
        return [self.unit_embed] + self.unit_blocks + [self.unit_head]

    # dropout sites: 0 = embedding, 1 + 2i = attention probs of block i, 2 + 2i = MLP output
    site_embed = 0

    @staticmethod
    def site_attn(i):
        return 1 + 2 * i

    @staticmethod
    def site_mlp(i):
        return 2 + 2 * i

    def num_params(self):
        return sum(p.numel() for p in self.parameters())

    def _prepare_layer_buffers(self, N, like):
        """Under an engine that batches weight gradients (``rt.defer_wgrad``), the GEMM operands of
        every block's dW products live in layer-strided buffers [L, R*N, k] -- one row per block, in
        the order of the blocks' gradient slots in the flat buffer -- so a group of blocks is one
        strided-batched GEMM (parallel/wgrad.py); the row order follows the engine's slot order
        (``rt.wgrad_rows_reversed``).  X: ln_1 / ln_2 outputs, attention output, GELU
        output; dY: dqkv, d(x1), d(fc1 pre-activation), d(fc2 output).  R = 1, or the accumulation
        window when the engine takes window-wide weight gradients (``rt.wgrad_window()``): micro-step
        m then writes token rows [m*N, (m+1)*N) and the last one hands over all R*N rows.
        ~1 GB per window row at TinyGPT-A."""
        if not (getattr(self.rt, "defer_wgrad", False) and self.training and torch.is_grad_enabled()):
            self._lbufs, self._lbuf_key = None, None
            return
        win = self.rt.wgrad_window()
        pos, R = win if win is not None else (0, 1)
        L, d, F = self.cfg.n_layer, self.cfg.n_embd, 4 * self.cfg.n_embd
        key = (L, N, R, d, like.dtype, like.device)
        if self._lbuf_key != key:
            self._lbufs = None                       # free the old set before allocating the new one
            self.__dict__.pop("_lbuf_views", None)   # (their cached views too)
            mk = lambda k: torch.empty(L, R * N, k, dtype=like.dtype, device=like.device)  # noqa: E731
            self._lbufs = SimpleNamespace(h1=mk(d), o=mk(d), h2=mk(d), g=mk(F), dqkv=mk(3 * d), dx1=mk(d),
                                          df=mk(F), dm=mk(d))
            self._lbuf_key = key
        self._lbuf_win = (pos, R, N)
        self._lbuf_on = True

    def layer_buffer(self, i):
        """Views of block ``i``'s row of the layer-strided buffers (this micro-step's token rows), or
        None (immediate dW).  ``window``: dW is window-wide; ``full`` (at the window's last
        micro-step, else None): the row's views over all of the window's tokens."""
        b = self._lbufs
        if b is None or not getattr(self, "_lbuf_on", False):
            return None
        r = self.cfg.n_layer - 1 - i if getattr(self.rt, "wgrad_rows_reversed", True) else i
        pos, R, N = self._lbuf_win
        # the views of one (row, window position) never change while the buffers live: build them once
        # (eight slices per block per micro-step were host time of every eager step)
        ck = (r, pos, R, N, id(b))
        cache = self.__dict__.setdefault("_lbuf_views", {})
        out = cache.get(ck)
        if out is None:
            if len(cache) > 4 * self.cfg.n_layer * max(R, 1):
                cache.clear()
            out = SimpleNamespace(**{k: v[r, pos * N:(pos + 1) * N] for k, v in vars(b).items()})
            out.window = R > 1
            out.full = SimpleNamespace(**{k: v[r] for k, v in vars(b).items()}) if (R > 1 and pos == R - 1) else None
            cache[ck] = out
        return out

    def forward(self, idx, targets=None, return_logits=False):
        B, T = idx.shape
        assert T <= self.cfg.block_size, f"Sequence {T} exceeds block size {self.cfg.block_size}"
        self._cur_bt = (B, T)
        if not self.training:
            self.drop_p = 0.0
        else:
            self.drop_p = self.cfg.dropout
        if self.drop_p > 0 and self.rt.seed is None:
            raise RuntimeError("dropout needs a StepSeed on the runtime (engine.attach or rt.seed = ...)")
        self._lbuf_on = False
        self._next_amask = None
        self._prepare_layer_buffers(B * T, self.transformer["wte"].weight)
        anchor = torch.empty((), requires_grad=True)    # graph entry (CPU scalar, never updated)
        x = _EmbedFn.apply(anchor, idx, self)
        m = None
        for i in range(len(self.unit_blocks)):
            x, m = _BlockFn.apply(x, m, self, i)
        logits, loss = _HeadFn.apply(x, m, self, targets, return_logits)
        if targets is None:
            return logits.view(B, T, -1), None
        return (logits.view(B, T, -1) if return_logits else None), loss
