"""Loader for the in-tree gfx950 kernel extension (<repo>/_so/_hip_kernels.so, _build.py).

GPU tensors always go through the HIP kernels: if the extension is missing on a
machine with a GPU, ``ext()`` raises instead of silently falling back to
PyTorch eager ops.
"""
from __future__ import annotations

import os

_EXT = None
_ERR = None


def ext():
    global _EXT, _ERR
    if _EXT is not None:
        return _EXT
    from .. import _build
    try:
        m = _build.load_hip()
    except ImportError as e:  # pragma: no cover - depends on build state
        _ERR = e
        if os.environ.get("FEDDDOS_AUTOBUILD", "1") == "1":
            _build.build_hip()
            m = _build.load_hip()
        else:
            raise RuntimeError(
                "gfx950 kernel extension is not built; run "
                "`python -m detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd._build`"
            ) from e
    _EXT = m
    return _EXT


def available() -> bool:
    try:
        ext()
        return True
    except Exception:
        return False


def so_path() -> str:
    return ext().__file__
