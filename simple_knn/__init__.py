"""Import shim: ``from simple_knn._C import distCUDA2`` (scene/gaussian_model.py:9) resolves to the
MI355X implementation in rain_amd.simple_knn."""
from rain_amd.simple_knn import _C  # noqa: F401
from rain_amd.simple_knn._C import distCUDA2  # noqa: F401
