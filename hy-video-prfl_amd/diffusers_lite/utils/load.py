# import path of the reference (diffusers_lite/utils/load.py); implementation: prfl_amd.fsdp_utils
from prfl_amd.fsdp_utils import get_no_split_modules  # noqa: F401
