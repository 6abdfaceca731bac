"""MI355X replacement of the reference's ``simple_knn`` extension (submodules/simple-knn,
imported by scene/gaussian_model.py:9 as ``from simple_knn._C import distCUDA2``)."""
from ._C import distCUDA2  # noqa: F401
