from prfl_amd.train import batch2list, list2batch  # noqa: F401
