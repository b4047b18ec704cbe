"""Loader for the in-tree ``dltb._C`` HIP extension (built by ``csrc/build.py`` for gfx950).

GPU code paths call :func:`ext` which raises loudly when the extension is missing — there is no
silent eager fallback on the GPU.  The torch reference implementations in :mod:`dltb.ops.ref`
serve CPU tests only.  ``DLTB_EXT_PATH`` loads another build of the same module instead (the
checked ``csrc/build.py --debug`` extension).
"""
import importlib
import importlib.util
import os
import sys

_C = None
_ERR = None


def _try_load():
    global _C, _ERR
    if _C is not None or _ERR is not None:
        return
    try:
        import torch  # noqa: F401  (libtorch must be loaded before the extension)
        name = __package__.rsplit(".", 1)[0] + "._C"
        alt = os.environ.get("DLTB_EXT_PATH")
        if alt:
            spec = importlib.util.spec_from_file_location(name, alt)
            _C = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(_C)
            sys.modules[name] = _C
        else:
            _C = importlib.import_module(name)
    except Exception as e:  # pragma: no cover - depends on the build
        _ERR = e


def available() -> bool:
    _try_load()
    return _C is not None


def ext():
    """Return the loaded extension or raise with build instructions."""
    _try_load()
    if _C is None:
        raise RuntimeError(
            "dltb._C (gfx950 HIP kernels) is not built or failed to load: "
            f"{_ERR!r}. Build it with `python csrc/build.py` (or __graft_entry__.build()).")
    return _C


def so_path():
    _try_load()
    return getattr(_C, "__file__", None) if _C is not None else None


def build_if_missing():
    """Build the extension in-tree when it is absent (used by the harness on GPU boxes)."""
    if available():
        return True
    import sys
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, os.path.join(root, "csrc"))
    try:
        import build as _b  # csrc/build.py
        _b.build(verbose=True)
    finally:
        sys.path.pop(0)
    global _ERR
    _ERR = None
    return available()
