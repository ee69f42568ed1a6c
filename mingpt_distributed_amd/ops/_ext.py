"""Loader for the in-tree gfx950 extension ``mingpt_distributed_amd/_C.so``.

GPU code paths call :func:`ext` which raises loudly if the extension is missing: there is no
silent eager fallback for a GPU tensor.  CPU tensors never reach the extension.

Debug mode: ``MINGPT_DEBUG_CHECKS=1`` wraps every extension entry point so the
device is synchronised after it and a HIP error or a device range-check hit is raised *at that
op*, named (the launch-blocking analogue).  With the ``-DMG_DEBUG`` build
(``python build_ext.py --debug``, ``MINGPT_EXT_SO=build/debug/_C.so``) the kernels also
range-check token ids and targets, clamp bad ones (no fault) and report them here.
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


_ERR_BITS = {1: "embedding_fwd: token id outside [0, vocab)",
             2: "embedding_bwd: token id outside [0, vocab)",
             4: "cross-entropy: target >= vocab"}


class DeviceCheckError(RuntimeError):
    """A device-side range check (MG_DEBUG build) or a HIP error, attributed to one op."""


class _Checked:
    """Extension proxy: synchronise after each call and raise on HIP errors / range-check bits."""

    def __init__(self, mod):
        self._mod = mod

    def __getattr__(self, name):
        fn = getattr(self._mod, name)
        if not callable(fn) or name in ("debug_error_bits", "debug_build"):
            return fn
        mod = self._mod

        def checked(*args, **kw):
            import torch

            out = fn(*args, **kw)
            if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
                # inside a hipGraph capture (StepEngine.graph_step) a sync or a blocking read
                # would invalidate the capture: the launch is checked when the graph replays
                return out
            try:
                torch.cuda.synchronize()
            except RuntimeError as e:
                raise DeviceCheckError(f"{name}: HIP error after the launch: {e}") from e
            bits = int(mod.debug_error_bits())
            if bits:
                what = "; ".join(m for b, m in _ERR_BITS.items() if bits & b)
                raise DeviceCheckError(f"{name}: device range check failed ({what})")
            return out

        return checked


def available() -> bool:
    _load()
    return _EXT is not None


def ext():
    _load()
    if _EXT is None:
        raise RuntimeError(
            "mingpt_distributed_amd._C (the gfx950 HIP extension) is not built or failed to load: "
            f"{_ERR!r}. Run `python build_ext.py` (hipcc --offload-arch=gfx950).")
    if os.environ.get("MINGPT_DEBUG_CHECKS", "0") not in ("", "0"):
        return _Checked(_EXT)
    return _EXT


def so_path() -> str:
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_C.so")
