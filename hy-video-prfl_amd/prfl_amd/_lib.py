"""ctypes binding of libprfl_hip.so (the C ABI declared in include/prfl_hip.h).

There is no CPU fallback: if the library or a GPU is missing, every op raises.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PRFL_HIP_LIB", os.path.join(_HERE, "lib", "libprfl_hip.so"))

P = ctypes.c_void_p
I64 = ctypes.c_int64
I32 = ctypes.c_int
F32 = ctypes.c_float

# name -> argtypes (mirrors include/prfl_hip.h)
SIGNATURES = {
    "prfl_gemm_bf16": [P, I64, I32, P, I64, I32, P, I64, I64, I64, I64, I32, P, P, P, I64, I32, P,
                       I64, I32, P],
    "prfl_gemm_bf16_tiled": [P, I64, I32, P, I64, I32, P, I64, I64, I64, I64, I32, P, P, P, I64,
                             I32, P, I64, I32, I32, P],
    "prfl_attn_fwd": [P, I64, I64, P, I64, I64, P, I64, I64, P, I64, I64, P, I64, I64, I64, I64,
                      I64, F32, P],
    "prfl_attn_fwd_ws": [P, I64, I64, P, I64, I64, P, I64, I64, P, I64, I64, P, I64, I64, I64, I64,
                         I64, F32, P, I64, P],
    "prfl_attn_fwd_ws_bytes": [I64, I64, I64, I64, I64],
    "prfl_attn_fwd_l2q_ws": [P, I64, I64, P, I64, I64, P, I64, I64, P, I64, I64, P, I64, I64, I64,
                             I64, I64, P, I64, P],
    "prfl_attn_vt_bytes": [I64, I64, I64],
    "prfl_attn_v_to_vt": [P, I64, I64, P, I64, I64, I64, P],
    "prfl_attn_fwd_l2q_vt_ws": [P, I64, I64, P, I64, I64, P, P, I64, I64, P, I64, I64, I64, I64, I64,
                                P, I64, P],
    "prfl_attn_fwd_fp8": [P, I64, I64, P, I64, I64, P, I64, I64, P, I64, I64, P, I64, I64, I64,
                          I64, I64, F32, P, I64, P],
    "prfl_attn_fwd_fp8_ws_bytes": [I64, I64, I64, I64, I64],
    "prfl_attn_fwd_fp8_l2q": [P, I64, I64, P, I64, I64, P, I64, I64, P, I64, I64, P, I64, I64, I64,
                              I64, I64, P, I64, P],
    "prfl_attn_bwd_ws": [P, I64, I64, P, I64, I64, P, I64, I64, P, I64, I64, P, I64, I64, P, P, P,
                         I64, I64, P, I64, I64, P, I64, I64, I64, I64, I64, I64, I64, F32, P, I64,
                         P],
    "prfl_attn_bwd_ws_bytes": [I64, I64, I64, I64, I64],
    "prfl_attn_bwd_l2q_ws": [P, I64, I64, P, I64, I64, P, I64, I64, P, I64, I64, P, I64, I64, P, P,
                             P, I64, I64, P, I64, I64, P, I64, I64, I64, I64, I64, I64, I64, P, I64,
                             P],
    "prfl_attn_bwd_l2q_kt_ws": [P, I64, I64, P, I64, I64, P, P, I64, I64, P, I64, I64, P, I64, I64,
                                P, P, P, I64, I64, P, I64, I64, P, I64, I64, I64, I64, I64, I64,
                                I64, P, I64, P],
    "prfl_attn_bwd": [P, I64, I64, P, I64, I64, P, I64, I64, P, I64, I64, P, I64, I64, P, P, P, I64,
                      I64, P, I64, I64, P, I64, I64, I64, I64, I64, I64, I64, F32, P],
    "prfl_ln_mod_fwd": [P, I32, I64, I64, I64, P, P, P, P, F32, P, I64, P, P, P],
    "prfl_ln_mod_bwd": [P, I64, P, I32, I64, P, P, I64, I64, P, P, P, I64, I32, P, P, P],
    "prfl_norm_rows_per_part": [],
    "prfl_rms_rope_fwd_scaled": [P, I64, I64, I64, P, F32, P, I64, I64, I64, P, I64, P, F32, P],
    "prfl_rms_rope_bwd_scaled": [P, I64, P, I64, P, I64, I64, P, P, I64, I64, I64, P, I64, P, F32,
                                 P],
    "prfl_rms_rope_fwd_pos": [P, I64, I64, I64, P, F32, P, I64, I64, I64, I64, P, I64, P, F32, P],
    "prfl_rms_rope_bwd_pos": [P, I64, P, I64, P, I64, I64, P, P, I64, I64, I64, I64, P, I64, P, F32,
                              P],
    "prfl_cast_f32_bf16": [P, P, I64, P],
    "prfl_cast_f32_bf16_t": [P, I64, I64, I64, P, I64, P],
    "prfl_gate_bwd": [P, I64, P, I64, P, I64, I64, P, I64, P, P, P],
    "prfl_colsum_bf16": [P, I64, I64, I64, P, P],
    "prfl_colsum_reduce": [P, I64, I64, P, I32, P],
    "prfl_colsum_rows_per_part": [],
    "prfl_sumsq": [P, I64, P, P],
    "prfl_scale": [P, I64, P, P],
    "prfl_adamw": [P, P, P, P, I64, F32, F32, F32, F32, F32, I64, P],
    "prfl_adamw_zero_grad": [P, P, P, P, I64, F32, F32, F32, F32, F32, I64, P],
    "prfl_quant_rows_fp8": [P, I32, I64, I64, I64, P, I64, P, P],
    "prfl_gemm_fp8": [P, I64, P, P, I64, P, P, I64, I64, I64, I64, I32, P, P, P, I64, I32, P, I64,
                      P],
    "prfl_unipc_step": [P, P, P, P, P, P, P, P, I64, P, I32, I32, P],
    "prfl_unipc_step_bwd": [P, P, I64, P, I32, I32, P],
    "prfl_query_pool_splits": [I64, I64, I64],
    "prfl_query_pool_fwd": [P, I64, P, I64, I64, I64, I64, I64, I64, F32, P, I64, P, P, P, P, P, I64,
                            P],
    "prfl_query_pool_bwd": [P, P, I64, P, I64, I64, P, P, I64, I64, I64, I64, F32, P, I64, P, I64,
                            I64, P, I64, P],
    "prfl_prof_enable": [I32],
    "prfl_prof_collect": [P, P, P, I32],
    "prfl_prof_clock": [P, P, P, P],
}

# entries that return a value other than a hipError_t code
RESTYPES = {"prfl_attn_fwd_ws_bytes": I64, "prfl_attn_vt_bytes": I64, "prfl_attn_fwd_fp8_ws_bytes": I64, "prfl_attn_bwd_ws_bytes": I64}

# kernel ids of the profiling hooks (csrc/common.h)
KID = dict(gemm=0, attn_fwd=1, attn_fwd_short=2, attn_bwd_dkdv=3, attn_bwd_dq=4, ln=5, rms=6,
           eltwise=7, adamw=8, pool=9, attn_fwd_fp8=10)
NKID = 11

_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"prfl_amd: HIP library not built ({LIB_PATH}); "
                               "run `make -C hy-video-prfl_amd`")
        lib = ctypes.CDLL(LIB_PATH)
        for name, args in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = RESTYPES.get(name, I32)
        _lib = lib
    return _lib


def call(name, *args):
    rc = getattr(load(), name)(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed with hipError {rc}")
    return rc


def stream_ptr(device=None):
    return P(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return P(0) if t is None else P(t.data_ptr())


def require_gpu(*tensors):
    for t in tensors:
        if t is not None and (not t.is_cuda):
            raise RuntimeError("prfl_amd ops run only on the MI355X (HIP) device; got a CPU tensor")
