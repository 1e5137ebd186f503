"""ctypes binding of libmmu_hip.so (the C-ABI declared in include/mmu.h).

The product path has no CPU fallback: if the library is missing or cannot be
loaded, or the tensors are not on a HIP device, calls raise immediately.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MMU_LIB_PATH: load another build of the same ABI (A/B timing of two kernel versions,
# tools/ab_build.sh); the default is the in-tree build
LIB_PATH = os.environ.get("MMU_LIB_PATH") or os.path.join(_HERE, "libmmu_hip.so")

c_i64, c_i32, c_f32, c_u64, c_vp = ctypes.c_int64, ctypes.c_int32, ctypes.c_float, ctypes.c_uint64, ctypes.c_void_p
c_f32p, c_i64p, c_dp = ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double)

MMU_BF16, MMU_F32 = 0, 1
(EPI_STORE, EPI_BIAS_GELU, EPI_BIAS_DROP_RES, EPI_DGELU, EPI_ADD_RES, EPI_BIAS_DROP_QGELU, EPI_STORE_STATS,
 EPI_STORE_BNB, EPI_ADD_RES_BNB) = range(9)


class Epilogue(ctypes.Structure):
    """mirror of ``mmu_epilogue`` (include/mmu.h)"""
    _fields_ = [("kind", c_i32), ("accumulate", c_i32), ("bias", c_vp), ("bias_bstride", c_i64),
                ("residual", c_vp), ("ldr", c_i64), ("res_bstride", c_i64), ("aux", c_vp), ("ldx", c_i64),
                ("aux_bstride", c_i64), ("colsum", c_vp), ("colsum_bstride", c_i64), ("drop_p", c_f32),
                ("seed", c_u64), ("workspace", c_vp), ("workspace_floats", c_i64), ("res_ln_mean", c_vp),
                ("res_ln_rstd", c_vp), ("res_ln_w", c_vp), ("res_ln_b", c_vp), ("res_ln_bstride", c_i64),
                ("bn_x", c_vp), ("bn_mask", c_vp), ("bn_mean", c_vp), ("res_mask", c_vp)]


# name -> (restype, argtypes); every entry must be exported by the library (tested on CPU)
SIGNATURES = {
    "mmu_version": (c_i32, []),
    "mmu_embed_bwd_ws_floats": (c_i64, [c_i64, c_i64, c_i64]),
    "mmu_last_error": (ctypes.c_char_p, []),
    "mmu_set_seed_offset": (c_i32, [c_vp]),
    "mmu_gemm": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_i64, c_i32, c_vp, c_i64, c_i32, c_i64, c_i64, c_i64,
                         c_i64, c_i64, c_i64, c_i64, ctypes.POINTER(Epilogue), c_vp]),
    "mmu_colsum_reduce": (c_i32, [c_vp, c_i64, c_i64, c_vp, c_i32, c_vp]),
    "mmu_colsum_reduce_multi": (c_i32, [c_i32, c_vp, c_vp, c_vp, c_i64, c_i32, c_vp]),
    "mmu_colsum_bf16": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_i32, c_vp]),
    "mmu_transpose_bf16_batched": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_vp]),
    "mmu_attention_fwd": (c_i32, [c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, c_i64, c_f32, c_u64, c_vp,
                                  c_vp]),
    "mmu_attention_bwd": (c_i32, [c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64,
                                  c_i64, c_i64, c_i64, c_f32, c_u64, c_vp, c_vp, c_vp]),
    "mmu_layernorm_fwd": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_f32, c_i64, c_i64, c_vp]),
    "mmu_layernorm_bwd": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_u64, c_vp, c_vp, c_vp,
                                  c_i64, c_i64, c_i64, c_vp]),
    "mmu_layernorm_fwd_f32": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_f32, c_i64, c_i64,
                                      c_vp]),
    "mmu_layernorm_bwd_f32": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_u64, c_vp, c_vp, c_vp,
                                      c_i64, c_i64, c_i64, c_vp]),
    "mmu_layernorm_bwd_res": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64,
                                      c_i64, c_vp]),
    "mmu_seqattn_fwd": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp]),
    "mmu_seqattn_bwd": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64,
                                c_i64, c_vp]),
    "mmu_embed_fwd": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_i64, c_i64, c_vp,
                              c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_f32, c_f32, c_u64, c_vp, c_vp, c_vp, c_vp,
                              c_vp, c_vp]),
    "mmu_embed_bwd": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64,
                              c_i64, c_i64, c_i64, c_f32, c_f32, c_u64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                              c_vp]),
    "mmu_image_normalize": (c_i32, [c_vp, c_i64, c_f32p, c_f32p, c_vp, c_i32, c_vp]),
    "mmu_maxpool_fwd": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "mmu_maxpool_bwd": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp]),
    "mmu_row_pool_fwd": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp]),
    "mmu_row_pool_bwd": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp]),
    "mmu_conv3x3_implicit": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp]),
    "mmu_conv3x3_implicit_bnb": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp,
                                         c_vp, c_vp, c_i64, c_vp]),
    "mmu_conv3x3_wgrad": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_vp, c_i64, c_vp]),
    "mmu_conv_implicit": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_i64,
                                  c_vp]),
    "mmu_conv_implicit_stats": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp,
                                        c_i64, c_vp]),
    "mmu_conv_wgrad": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_vp, c_i64,
                               c_vp]),
    "mmu_stem_conv_fwd": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp]),
    "mmu_stem_conv_wgrad_ws_floats": (c_i64, [c_i64, c_i64, c_i64]),
    "mmu_stem_conv_wgrad": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i32, c_vp, c_i64, c_vp]),
    "mmu_batchnorm_ws_bytes": (c_i64, [c_i64]),
    "mmu_batchnorm_fwd": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_f32,
                                  c_f32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "mmu_batchnorm_bwd": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp,
                                  c_vp, c_vp, c_vp, c_i64, c_vp]),
    "mmu_batchnorm_bwd_parts": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_i32,
                                        c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "mmu_batchnorm_stats": (c_i32, [c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp]),
    "mmu_batchnorm_fwd_sums": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32,
                                       c_f32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "mmu_batchnorm_fwd_parts": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                        c_f32, c_f32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "mmu_batchnorm_bwd_reduce": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp,
                                         c_vp, c_i64, c_vp]),
    "mmu_batchnorm_bwd_sums": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp,
                                       c_vp, c_vp, c_i64, c_vp]),
    "mmu_bertadam_step": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_f32, c_f32, c_f32,
                                  c_f32, c_f32, c_f32, c_f32, c_f32, c_f32, c_f32, c_vp, c_i64, c_vp]),
    "mmu_uncertainty": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mmu_ece_bins": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp]),
    "mmu_timing_enable": (c_i32, [c_i32]),
    "mmu_timing_pause": (c_i32, [c_i32]),
    "mmu_timing_read": (c_i32, [c_dp, c_i64p, c_dp]),
}

_lib = None


class NativeError(RuntimeError):
    pass


# include/mmu.h MMU_ABI_VERSION: the argument lists SIGNATURES binds
ABI_VERSION = 4


def load():
    """Load (once) and return the library; raise NativeError if it is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(f"libmmu_hip.so not built at {LIB_PATH}: run `python -c 'import __graft_entry__ as g; "
                              f"g.build()'` (hipcc --offload-arch=gfx950)")
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()  # let torch own HIP runtime / context creation before our code object registers
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        if lib.mmu_version() != ABI_VERSION:
            raise NativeError(f"libmmu_hip.so ABI {lib.mmu_version()} != {ABI_VERSION} (include/mmu.h "
                              "MMU_ABI_VERSION): rebuild the library")
        _lib = lib
    return _lib


def call(name, *args):
    rc = getattr(load(), name)(*args)
    if rc != 0:
        raise NativeError(f"{name}: {load().mmu_last_error().decode()}")
    return rc


def last_error():
    return load().mmu_last_error().decode()
