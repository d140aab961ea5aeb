from .attention import flash_attention, attention  # noqa: F401
from .model import WanModel  # noqa: F401
