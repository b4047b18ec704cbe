"""hipBLASLt GEMM selection via PyTorch TunableOp.

The plain library GEMMs of the model (QKV / out / fc1 / fc2 projections, the tied head, and their
dX / dW products) run on hipBLASLt.  Its default heuristic picks mediocre solutions for the
M = B*T = 2048 training shapes, so the framework ships TunableOp results measured on MI355X
(``configs/tunableop/*.csv``) and enables them at start-up:

    mode "use"  (default when a results file exists): replay the shipped solutions, no tuning
    mode "tune" : benchmark every hipBLASLt/rocBLAS candidate for each new GEMM signature and write
                  the results file (run once on one GPU; ``scripts/tune_gemms.sh``)
    mode "off"  : library defaults

On top of TunableOp's solution choice, "use" also loads the hipBLASLt extension-API table
(``configs/blaslt/*.csv``, :mod:`dltb.ops.blaslt`): per exact problem a solution plus run-time
split-K and workgroup mapping, measured faster than TunableOp's pick by ``scripts/tune_blaslt.py``.
The returned mode string then reads ``use+blaslt<n entries>``.
"""
import os

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DEFAULT_FILE = os.path.join(_ROOT, "configs", "tunableop", "tunableop_results_gfx950.csv")


def setup_tunableop(mode: str = "auto", path: str = None, verbose: bool = False) -> str:
    import torch
    if not torch.cuda.is_available() or mode == "off":
        return "off"
    try:
        import torch.cuda.tunable as tn
    except Exception:
        return "unavailable"
    path = path or os.environ.get("DLTB_TUNABLEOP_FILE", DEFAULT_FILE)
    if mode == "auto":
        mode = "use" if os.path.exists(path) else "off"
    if mode == "off":
        return "off"
    tn.enable(True)
    tn.set_filename(path, False)
    if mode == "tune":
        os.makedirs(os.path.dirname(path), exist_ok=True)
        tn.tuning_enable(True)
        tn.set_max_tuning_duration(int(os.environ.get("DLTB_TUNE_MS", "60")))
        tn.set_max_tuning_iterations(int(os.environ.get("DLTB_TUNE_ITERS", "100")))
    else:
        tn.tuning_enable(False)
        tn.read_file(path)
    if verbose:
        print(f"[dltb] TunableOp {mode}: {path}", flush=True)
    if mode == "use":
        from ..ops import blaslt
        n = blaslt.load(verbose=verbose)
        if n:
            return f"use+blaslt{n}"
    return mode


def flush_tunableop():
    try:
        import torch.cuda.tunable as tn
        if tn.is_enabled() and tn.tuning_is_enabled():
            tn.write_file()
    except Exception:
        pass
