from prfl_amd.data import (BlockDistributedSampler, align_floor_to, crop_tensor,  # noqa: F401
                           LatentPrefetcher)
