"""Import-path shim: the reference's `diffusers_lite` hot-path modules, served by prfl_amd.

Scripts written against Tencent-Hunyuan/HY-Video-PRFL (`from diffusers_lite.wan.modules.model
import WanModel`, `from diffusers_lite.utils.network import QueryAttention, MLP, forward_mlp`, ...)
resolve to the MI355X-native implementations when `hy-video-prfl_amd/` is on sys.path.
Only the PRFL/PAVRM hot path is provided; VAE/T5/CLIP/inference pipelines are not.
"""
