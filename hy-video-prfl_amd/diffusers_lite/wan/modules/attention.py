from prfl_amd.attention import attention, flash_attention  # noqa: F401
