from prfl_amd.data import Image2VideoTrainDataset  # noqa: F401
