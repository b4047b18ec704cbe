"""Tuned hipBLASLt GEMMs: (solution, split-K, workgroup mapping) per problem, from a shipped table.

TunableOp (``utils/gemm_tuning.py``) picks the fastest hipBLASLt *solution* per GEMM signature,
but each solution runs with its compiled-in split-K and workgroup-to-tile mapping.  hipBLASLt's
extension API takes both as run-time parameters (``hipblaslt_ext::GemmTuning``), and they matter
most for exactly the products a 2048-token micro-batch produces: a [2048 x 1024] output is 128-256
tiles, one partial wave on 256 CUs, so the split of K decides how full the machine is and the
mapping decides which A/B panels an XCD's 4 MB L2 shares.  ``scripts/tune_blaslt.py`` records the
model's GEMM problems (exact shapes, strides, accumulate flag), times every solution and the best
ones under a (split-K x wgm) grid, and writes ``configs/blaslt/blaslt_gfx950.csv``; at run time
:func:`mm` hands the product to ``dltb._C.blaslt_mm``, which forms the key, looks it up in the
table (held in C++) and runs the stored triple (csrc/blaslt.cpp) -- a few microseconds of host time
against ~25 us for a torch matmul with TunableOp -- otherwise it returns False and the caller keeps
its torch / TunableOp path.

Problems are keyed in column-major BLAS terms.  A row-major torch product C[M, N] = A[M, K] B[K, N]
is the column-major C^T = B^T A^T: BLAS m = N, n = M, k = K, BLAS "A" = torch B, BLAS "B" = torch A.
Batched products (``[b, M, K] @ [b, K, N]`` on strided views) add the batch strides.
"""
import csv
import os
from typing import Dict, Optional, Tuple

import torch

from ._ext import ext

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DEFAULT_FILE = os.path.join(_ROOT, "configs", "blaslt", "blaslt_gfx950.csv")
FIELDS = ["dtype", "opA", "opB", "m", "n", "k", "batch", "lda", "ldb", "ldc", "sa", "sb", "sc", "beta1", "bias",
          "algo", "splitk", "wgm", "us", "torch_us", "solution"]

Key = Tuple

_table: Dict[Key, Tuple[int, int, int]] = {}
_enabled = False
_recording: Optional[dict] = None


def _operand(t: torch.Tensor):
    """(op, ld) of the BLAS operand t^T (torch B as BLAS A, torch A as BLAS B): op N when the rows
    of ``t`` are contiguous (t^T is then column-major), op T when ``t`` itself is column-major.
    None when neither inner stride is 1."""
    s0, s1 = t.stride(-2), t.stride(-1)
    r, c = t.shape[-2], t.shape[-1]
    if s1 == 1 and (s0 >= c or r == 1):       # rows of t contiguous: t^T is column-major, op N
        return 0, max(s0, c)
    if s0 == 1 and (s1 >= r or c == 1):       # t itself column-major: op T
        return 1, max(s1, r)
    return None


def problem(a: torch.Tensor, b: torch.Tensor, c: torch.Tensor, accumulate: bool, bias=None) -> Optional[Key]:
    """BLAS key of ``c (+)= a @ b (+ bias)`` (2-D, or 3-D batched) or None if it cannot be expressed."""
    if a.dim() != b.dim() or a.dim() != c.dim() or a.dim() not in (2, 3):
        return None
    if c.stride(-1) != 1 or a.dtype != b.dtype or a.dtype != c.dtype or a.dtype not in (torch.bfloat16, torch.float16):
        return None
    M, K = a.shape[-2], a.shape[-1]
    N = b.shape[-1]
    if b.shape[-2] != K or c.shape[-2] != M or c.shape[-1] != N:
        return None
    if bias is not None and (a.dim() != 2 or accumulate or bias.dtype != a.dtype or not bias.is_contiguous()
                             or bias.numel() != N):
        return None
    oa, ob = _operand(b), _operand(a)
    if oa is None or ob is None:
        return None
    batch = a.shape[0] if a.dim() == 3 else 1
    sa = b.stride(0) if a.dim() == 3 else 0
    sb = a.stride(0) if a.dim() == 3 else 0
    sc = c.stride(0) if a.dim() == 3 else 0
    ldc = max(c.stride(-2), N)
    dt = "bf16" if a.dtype == torch.bfloat16 else "fp16"
    return (dt, oa[0], ob[0], N, M, K, batch, oa[1], ob[1], ldc, sa, sb, sc, int(bool(accumulate)),
            int(bias is not None))


def resolve_config_path(path: str, what: str) -> str:
    """A table path as given, or relative to the repository root when the working directory does
    not hold it (profilers run bench.py from /tmp).  A named table that exists nowhere is an error:
    silently running without it would time a different configuration."""
    if path == "none" or os.path.isabs(path) or os.path.exists(path):
        if path != "none" and not os.path.exists(path):
            raise FileNotFoundError(f"{what}: {path} does not exist")
        return path
    alt = os.path.join(_ROOT, path)
    if not os.path.exists(alt):
        raise FileNotFoundError(f"{what}: {path} exists neither in {os.getcwd()} nor in {_ROOT}")
    return alt


def load(path: str = None, verbose: bool = False) -> int:
    """Read the tuning table (``DLTB_BLASLT_FILE`` or the shipped one); entries whose solution name
    no longer matches the loaded library are dropped.  Returns the number of usable entries."""
    global _enabled
    path = resolve_config_path(path or os.environ.get("DLTB_BLASLT_FILE", DEFAULT_FILE), "DLTB_BLASLT_FILE")
    _table.clear()
    _enabled = False
    if not torch.cuda.is_available():
        return 0
    ext().blaslt_table_set([])
    if path == "none" or not os.path.exists(path):
        return 0
    C = ext()
    dropped = 0
    with open(path) as f:
        for row in csv.DictReader(f):
            key = (row["dtype"],) + tuple(int(row[k]) for k in FIELDS[1:15])
            algo = int(row["algo"])
            if row.get("solution") and C.blaslt_name(algo) != row["solution"]:
                dropped += 1
                continue
            _table[key] = (algo, int(row["splitk"]), int(row["wgm"]))
    _enabled = bool(_table)
    C.blaslt_table_set([[1 if k[0] == "fp16" else 0, *k[1:], *v] for k, v in _table.items()])
    if verbose:
        print(f"[dltb] hipBLASLt tuned GEMMs: {len(_table)} entries from {path}"
              + (f" ({dropped} stale dropped)" if dropped else ""), flush=True)
    return len(_table)


def disable():
    global _enabled
    _enabled = False
    if torch.cuda.is_available():
        ext().blaslt_table_set([])


def enabled() -> bool:
    return _enabled


def active() -> bool:
    """True when :func:`mm` may act (table loaded, or the tuner is recording)."""
    return _enabled or _recording is not None


def start_recording():
    """Collect the GEMM problems :func:`mm` sees (tuner): key -> (a, b, c, accumulate, bias)."""
    global _recording
    _recording = {}


def stop_recording() -> dict:
    global _recording
    r, _recording = _recording, None
    return r or {}


def run(key: Key, a, b, c, entry, bias=None) -> None:
    algo, sk, wg = entry
    _, opA, opB, m, n, k, batch, lda, ldb, ldc, sa, sb, sc, beta1, _ = key
    # BLAS A = torch b, BLAS B = torch a
    ext().blaslt_run(b, a, c, opA, opB, m, n, k, batch, lda, ldb, ldc, sa, sb, sc, bool(beta1), bias, algo, sk, wg)


def mm(a: torch.Tensor, b: torch.Tensor, c: torch.Tensor, accumulate: bool = False, bias=None) -> bool:
    """``c (+)= a @ b (+ bias)`` with the tuned solution if the table has this problem; False
    otherwise (nothing was launched and the caller runs its own GEMM)."""
    if _recording is not None and a.is_cuda:
        key = problem(a, b, c, accumulate, bias)
        if key is not None and key not in _recording:
            _recording[key] = (a, b, c, accumulate, bias)
        return False
    if not (_enabled and a.is_cuda):
        return False
    return ext().blaslt_mm(a, b, c, bool(accumulate), bias)     # key + lookup + launch in C++
