"""Import shim for ``simple_knn._C`` (see simple_knn/__init__.py)."""
from rain_amd.simple_knn._C import distCUDA2  # noqa: F401
