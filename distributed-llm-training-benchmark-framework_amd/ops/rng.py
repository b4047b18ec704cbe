"""Counter-based dropout RNG shared bit-for-bit by the HIP kernels and the torch reference.

The reference model (``train_harness.py:53,116,122``) applies dropout p=0.1 to the embedding sum,
the attention probabilities and the MLP output, using cuRAND Philox.  A 10-round Philox per
attention-probability element costs more VALU than the attention math itself on CDNA4 (D=64),
so the MI355X kernels use a cheaper counter hash instead:

    row_key = fmix32(row * 0x9E3779B1 + seed_hi)
    x       = fmix32(row_key ^ ((col >> 1) * 0x85EBCA77 + seed_lo))
    r16     = (col & 1) ? x >> 16 : x & 0xFFFF
    keep    = r16 >= thr16,   thr16 = round(p * 65536)

``fmix32`` is the MurmurHash3 finaliser (a bijective avalanche mixer).  One hash yields the
decisions for two adjacent columns and ``row_key`` is hoisted per row.  The attention-probability
mask (T x T decisions per head) uses :func:`attn_keep_mask`, which mixes the column key on its own and
combines the two keys with one multiply-xorshift round (3 VALU ops per column pair instead of 6).  Every dropout site views its tensor as ``[rows, cols]`` and
gets its own 64-bit seed ``site_seed(step_seed, site)``; the backward kernels regenerate the
identical mask instead of storing it.
"""
import torch

MASK32 = 0xFFFFFFFF
C_ROW = 0x9E3779B1
C_COL = 0x85EBCA77
GOLDEN64 = 0x9E3779B97F4A7C15


def splitmix64(x: int) -> int:
    x = (x + GOLDEN64) & 0xFFFFFFFFFFFFFFFF
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)


def site_seed(step_seed: int, site: int) -> int:
    """64-bit seed of one dropout site; identical to ``dltb_site_seed`` in csrc/common.h."""
    return splitmix64((step_seed + site * GOLDEN64) & 0xFFFFFFFFFFFFFFFF)


def drop_threshold(p: float) -> int:
    return min(65536, int(p * 65536.0 + 0.5))


def _mul32(a: torch.Tensor, c: int) -> torch.Tensor:
    # (a * c) mod 2^32 without overflowing signed int64
    lo = a * (c & 0xFFFF)
    hi = ((a * (c >> 16)) & 0xFFFF) << 16
    return (lo + hi) & MASK32


def _fmix32(h: torch.Tensor) -> torch.Tensor:
    h = h ^ (h >> 16)
    h = _mul32(h, 0x85EBCA6B)
    h = h ^ (h >> 13)
    h = _mul32(h, 0xC2B2AE35)
    h = h ^ (h >> 16)
    return h


def keep_mask(seed: int, rows: torch.Tensor, cols: torch.Tensor, p: float) -> torch.Tensor:
    """Boolean keep-mask for broadcastable int64 ``rows``/``cols`` index tensors."""
    s_lo = seed & MASK32
    s_hi = (seed >> 32) & MASK32
    rk = _fmix32((_mul32(rows, C_ROW) + s_hi) & MASK32)
    x = _fmix32(rk ^ ((_mul32(cols >> 1, C_COL) + s_lo) & MASK32))
    r16 = torch.where((cols & 1) == 1, x >> 16, x & 0xFFFF)
    return r16 >= drop_threshold(p)


def attn_keep_mask(seed: int, rows: torch.Tensor, cols: torch.Tensor, p: float) -> torch.Tensor:
    """Keep-mask of the attention-probability dropout (csrc/common.h ``rng_attn_pair``): the same row key,
    the column-pair key mixed by its own ``fmix32``, and one multiply-xorshift round per (row, pair) --
    ``x = (rk ^ fmix32(ck)) * 0x85EBCA6B; x ^= x >> 16``.  Half the per-pair VALU of ``keep_mask`` for the
    T x T decisions per head, which dominate a step's dropout work."""
    s_lo = seed & MASK32
    s_hi = (seed >> 32) & MASK32
    rk = _fmix32((_mul32(rows, C_ROW) + s_hi) & MASK32)
    ck = _fmix32((_mul32(cols >> 1, C_COL) + s_lo) & MASK32)
    x = _mul32(rk ^ ck, 0x85EBCA6B)
    x = x ^ (x >> 16)
    r16 = torch.where((cols & 1) == 1, x >> 16, x & 0xFFFF)
    return r16 >= drop_threshold(p)


def keep_mask_2d(seed: int, n_rows: int, n_cols: int, p: float, device=None,
                 row_offset: int = 0) -> torch.Tensor:
    rows = torch.arange(row_offset, row_offset + n_rows, dtype=torch.int64, device=device)[:, None]
    cols = torch.arange(n_cols, dtype=torch.int64, device=device)[None, :]
    return keep_mask(seed, rows, cols, p)


def dropout_ref(x: torch.Tensor, p: float, seed: int) -> torch.Tensor:
    """Reference dropout of ``x`` viewed as [-1, x.shape[-1]] (training mode)."""
    if p <= 0.0:
        return x
    n_cols = x.shape[-1]
    keep = keep_mask_2d(seed, x.numel() // n_cols, n_cols, p, device=x.device).view(x.shape)
    return torch.where(keep, x * (1.0 / (1.0 - p)), torch.zeros((), dtype=x.dtype, device=x.device))


class StepSeed:
    """Per-process dropout seed source.

    Every micro-step draws a fresh 64-bit ``step_seed``; each dropout site derives its own seed with
    :func:`site_seed`.  The value is also mirrored into a 1-element int64 device tensor so that
    kernels (and HIP-graph replays) read it from device memory without host syncs.
    """

    def __init__(self, base_seed: int, rank: int = 0, device=None):
        self.state = splitmix64((base_seed * 1000003 + rank * 7919) & 0xFFFFFFFFFFFFFFFF)
        self.value = self.state
        self.device_tensor = None
        if device is not None and torch.device(device).type == "cuda":
            self.device_tensor = torch.zeros(1, dtype=torch.int64, device=device)

    def next(self) -> int:
        self.state = splitmix64(self.state)
        self.value = self.state
        if self.device_tensor is not None and not torch.cuda.is_current_stream_capturing():
            self.upload()
        return self.value

    def upload(self):
        """Mirror the current value into the device tensor (a graph runner calls this before each
        replay; inside a capture ``next`` only advances the host state)."""
        v = self.value - (1 << 64) if self.value >= (1 << 63) else self.value
        self.device_tensor.fill_(v)
