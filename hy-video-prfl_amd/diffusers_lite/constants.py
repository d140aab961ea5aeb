from prfl_amd.data import NULL_DIR  # noqa: F401
