from prfl_amd.schedulers import FlowUniPCMultistepScheduler  # noqa: F401
