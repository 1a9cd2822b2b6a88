"""Loader for the C++ text extension (data/_text_native_impl*.so); builds it on demand."""
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
    try:
        from . import _text_native_impl as m
    except ImportError:
        if os.environ.get("FEDDDOS_AUTOBUILD", "1") != "1":
            return None
        try:
            from .. import _build
            _build.build_text()
            from . import _text_native_impl as m  # noqa: F811
        except Exception:
            return None
    _MOD = m
    return _MOD
