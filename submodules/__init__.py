"""Zero-edit import path for the reference's callers (SURVEY §8(b) "Build / import").

gaussian_renderer/__init__.py:5 imports
``submodules.diff_gaussian_rasterization.diff_gaussian_rasterization``; with this repository on
``sys.path`` that dotted path resolves to the MI355X rasterizer in ``rain_amd`` (no JIT build runs:
the HIP libraries are built ahead of time by ``__graft_entry__.build()``).
"""
