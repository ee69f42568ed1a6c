"""Loader for the in-tree gfx950 extension ``mingpt_distributed_amd/_C.so``.

GPU code paths call :func:`ext` which raises loudly if the extension is missing: there is no
silent eager fallback for a GPU tensor.  CPU tensors never reach the extension.
"""
from __future__ import annotations

import importlib
import importlib.util
import os

_EXT = None
_ERR = None


def _load():
    global _EXT, _ERR
    if _EXT is not None or _ERR is not None:
        return
    try:
        import torch  # noqa: F401  (loads torch's HIP runtime first; _C.so binds to it)

        alt = os.environ.get("MINGPT_EXT_SO")  # A/B runs: another build of the same extension
        if alt:
            spec = importlib.util.spec_from_file_location("mingpt_distributed_amd._C", alt)
            _EXT = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(_EXT)
        else:
            _EXT = importlib.import_module("mingpt_distributed_amd._C")
    except Exception as e:  # pragma: no cover - depends on build state
        _ERR = e


def available() -> bool:
    _load()
    return _EXT is not None


def ext():
    _load()
    if _EXT is None:
        raise RuntimeError(
            "mingpt_distributed_amd._C (the gfx950 HIP extension) is not built or failed to load: "
            f"{_ERR!r}. Run `python build_ext.py` (hipcc --offload-arch=gfx950).")
    return _EXT


def so_path() -> str:
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_C.so")
