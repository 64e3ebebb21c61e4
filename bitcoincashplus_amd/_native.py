"""Loader for the in-tree native extension ``_bcpnative``.

The extension holds the whole C++ consensus core plus the host side of the
gfx950 HIP kernels.  It is built in-tree by ``make`` (see ``__graft_entry__.build``)
and never silently replaced by a Python fallback: if it is missing, importing
this module raises with the build command to run.

PyTorch (when importable) is imported first so that the process uses torch's
HIP runtime instance (same ``libamdhip64.so.7`` soname) — the kernels then share
devices/streams with ``torch.cuda`` and RCCL in the multi-GPU paths.
"""
from __future__ import annotations

import importlib
import os

try:  # share one HIP runtime with torch / RCCL
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is part of the image
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))

try:
    _alt = os.environ.get("BCP_NATIVE_PATH")
    if _alt:  # A/B benchmarking: load another build of the same extension (tools/ab_bench.py)
        import importlib.machinery
        import importlib.util
        _spec = importlib.util.spec_from_file_location(
            "bitcoincashplus_amd._bcpnative", _alt,
            loader=importlib.machinery.ExtensionFileLoader("bitcoincashplus_amd._bcpnative", _alt))
        native = importlib.util.module_from_spec(_spec)
        _spec.loader.exec_module(native)
    else:
        native = importlib.import_module("bitcoincashplus_amd._bcpnative")
except ImportError as e:  # pragma: no cover
    raise ImportError(
        "bitcoincashplus_amd native extension not built: run `make -j8` in "
        f"{os.path.dirname(_HERE)} (or python -c 'import __graft_entry__ as g; g.build()')"
    ) from e


def gpu_available() -> bool:
    return bool(native.gpu_available())


def require_gpu(what: str = "this operation") -> None:
    """Fail loudly instead of silently falling back to CPU."""
    if not native.gpu_available():
        raise RuntimeError(f"{what} needs a HIP device (MI355X / gfx950); none is visible")


def native_path() -> str:
    return native.__file__
