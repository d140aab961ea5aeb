"""prfl_amd — MI355X-native (gfx950) PRFL hot path: the Wan DiT forward/backward that drives the
generator denoising chain and the PAVRM latent reward head, on hand-written HIP kernels
(``lib/libprfl_hip.so``, C ABI in ``include/prfl_hip.h``)."""
__version__ = "0.1.0"
