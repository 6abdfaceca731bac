"""Reference package ``submodules/diff_gaussian_rasterization`` (see submodules/__init__.py)."""
