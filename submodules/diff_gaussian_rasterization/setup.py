"""Stands where the reference's setup.py is imported from (``from ..setup import _C``,
diff_gaussian_rasterization/__init__.py:4, setup.py:8-19 JIT-loads the CUDA sources there).  Here
``_C`` is the ahead-of-time-built MI355X extension; nothing is compiled on import."""
from rain_amd.diff_gaussian_rasterization import _C  # noqa: F401
