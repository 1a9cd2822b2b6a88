"""Compute ops: gfx950 HIP kernels (``kernels``), their torch reference (``reference``),
the dropout hash (``dropout``) and the fused autograd functions (``functional``)."""
from . import dropout, reference  # noqa: F401
from ._ext import available as hip_available, ext  # noqa: F401
