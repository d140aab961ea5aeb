from prfl_amd.schedulers import FlowMatchDiscreteScheduler  # noqa: F401
