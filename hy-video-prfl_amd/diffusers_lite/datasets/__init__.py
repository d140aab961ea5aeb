from .image2video_dataset import Image2VideoTrainDataset  # noqa: F401
