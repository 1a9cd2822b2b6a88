"""Loader for the C++ text extension (<repo>/_so/_text_native_impl.so, _build.py); builds it on demand."""
from __future__ import annotations

import os

_MOD = None
_TRIED = False


def load():
    """Return the native module, or None if it cannot be built/imported (pure-Python fallback)."""
    global _MOD, _TRIED
    if _MOD is not None or _TRIED:
        return _MOD
    _TRIED = True
    from .. import _build
    try:
        m = _build.load_text()
    except ImportError:
        if os.environ.get("FEDDDOS_AUTOBUILD", "1") != "1":
            return None
        try:
            _build.build_text()
            m = _build.load_text()
        except Exception:
            return None
    _MOD = m
    return _MOD
