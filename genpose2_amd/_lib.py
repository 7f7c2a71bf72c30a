"""ctypes binding of libgenpose_hip.so (include/genpose_hip.h).

The library is built in-tree (``genpose2_amd/libgenpose_hip.so``, see ``__graft_entry__.build``).
There is no fallback: if the library is missing or a call fails, a ``GenPoseHipError`` is raised.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Iterable

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GENPOSE_HIP_LIB", os.path.join(_HERE, "libgenpose_hip.so"))

c_int, c_float, c_size_t, c_void_p = ctypes.c_int, ctypes.c_float, ctypes.c_size_t, ctypes.c_void_p
c_double = ctypes.c_double
c_int64_p = ctypes.POINTER(ctypes.c_int64)
c_uint64 = ctypes.c_uint64


class GenPoseHipError(RuntimeError):
    pass


class HeadWeights(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in ("pe0_w", "pe0_b", "pe2_w", "pe2_b", "h1p_w", "h2_w", "h2_b",
                                       "h1pts_t", "h1_b", "gfp_w", "te_w_t", "te_b", "h1t_t", "pe2_h", "h1p_h",
                                       "hsc")]


class ScaleWeights(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in ("ae0_w", "ae0_b", "ae2_w", "ae2_b", "ft0_w", "ft0_b", "ft2_w",
                                       "ft2_b")]


# name -> (restype, argtypes)
_SIGS: Dict[str, tuple] = {
    "gp_last_error": (ctypes.c_char_p, []),
    "gp_abi_version": (c_int, []),
    "gp_furthest_point_sampling": (c_int, [c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gp_gather_points": (c_int, [c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gp_ball_query": (c_int, [c_int, c_int, c_int, c_float, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gp_group_points": (c_int, [c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gp_encoder_workspace_size": (c_size_t, [c_int, c_int]),
    "gp_encoder_workspace_layout": (c_int, [c_int, c_int, c_int64_p]),
    "gp_encoder_forward": (c_int, [c_void_p, c_int64_p, c_void_p, c_int, c_int, c_void_p, c_size_t, c_void_p,
                                   c_void_p]),
    "gp_encoder_fps": (c_int, [c_void_p, c_int, c_int, c_void_p, c_size_t, c_void_p]),
    "gp_encoder_geometry": (c_int, [c_void_p, c_int, c_int, c_void_p, c_size_t, c_void_p]),
    "gp_encoder_forward_geom": (c_int, [c_void_p, c_int64_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_size_t,
                                        c_void_p, c_void_p]),
    "gp_encoder_geometry_levels": (c_int, [c_void_p, c_int, c_int, c_void_p, c_size_t, c_int, c_int, c_void_p]),
    "gp_encoder_forward_geom_levels": (c_int, [c_void_p, c_int64_p, c_void_p, c_int, c_int, c_void_p, c_void_p,
                                               c_size_t, c_void_p, c_int, c_int, c_void_p]),
    "gp_sa_level": (c_int, [c_void_p, c_int64_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_size_t,
                            c_void_p, c_void_p]),
    "gp_sa_level_geom": (c_int, [c_void_p, c_int64_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p,
                                 c_void_p, c_size_t, c_void_p, c_void_p]),
    "gp_linear": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p]),
    "gp_linear_split_words": (c_size_t, [c_int, c_int]),
    "gp_linear_split": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int,
                                c_void_p, c_int, c_void_p, c_void_p]),
    "gp_add_layernorm": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_float, c_void_p, c_void_p,
                                 c_void_p]),
    "gp_relpe_bias_bytes": (c_size_t, [c_int, c_int]),
    "gp_relpe_bias": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "gp_mha_attention": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "gp_mha_relpe_attention": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                                       c_void_p]),
    "gp_interp_points": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "gp_fusion_attend_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "gp_fusion_attend": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                 c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "gp_fusion_mix": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "gp_weights_pack": (c_int, [c_int, c_int, c_void_p, c_void_p, c_void_p, ctypes.POINTER(c_void_p)]),
    "gp_weights_free": (None, [c_void_p]),
    "gp_weights_heads": (ctypes.POINTER(HeadWeights), [c_void_p]),
    "gp_weights_scale": (ctypes.POINTER(ScaleWeights), [c_void_p]),
    "gp_weights_encoder": (c_void_p, [c_void_p, ctypes.POINTER(c_int64_p)]),
    "gp_weights_pack_host": (c_int, [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                     ctypes.POINTER(c_size_t), c_int64_p, c_int64_p]),
    "gp_head_object_proj": (c_int, [ctypes.POINTER(HeadWeights), c_void_p, c_int, c_void_p, c_void_p]),
    "gp_head_time_proj": (c_int, [ctypes.POINTER(HeadWeights), c_void_p, c_int, c_void_p, c_void_p]),
    "gp_score_eval": (c_int, [ctypes.POINTER(HeadWeights), c_void_p, c_void_p, c_float, c_void_p, c_int, c_int,
                              c_void_p, c_void_p]),
    "gp_energy_eval": (c_int, [ctypes.POINTER(HeadWeights), c_void_p, c_void_p, c_float, c_void_p, c_int, c_int,
                               c_void_p, c_void_p]),
    "gp_pc_workspace_size": (c_size_t, [c_int]),
    "gp_pc_tile_rows": (c_int, [c_int, c_int]),
    "gp_pc_sample": (c_int, [ctypes.POINTER(HeadWeights), c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int,
                             c_int, c_void_p, c_void_p, c_void_p, c_uint64, c_float, c_void_p, c_void_p, c_void_p,
                             c_void_p, c_size_t, c_void_p]),
    "gp_pc_global_partials": (c_int, [c_int, c_int, c_int, c_int]),
    "gp_pc_sample_global": (c_int, [ctypes.POINTER(HeadWeights), c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int,
                                    c_int, c_void_p, c_uint64, c_float, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                    c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "gp_pose_epilogue_f64": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "gp_ode_workspace_size": (c_size_t, [c_int]),
    "gp_ode_rhs": (c_int, [ctypes.POINTER(HeadWeights), c_void_p, c_float, c_float, c_double, c_void_p, c_void_p,
                           c_void_p, c_int, c_double, c_int, c_int, c_void_p, c_void_p, c_size_t, c_void_p]),
    "gp_ode_attempt": (c_int, [ctypes.POINTER(HeadWeights), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_void_p, c_void_p, c_double, c_double, c_double, c_int, c_int,
                               c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "gp_ode_init_norms": (c_int, [c_void_p, c_void_p, c_void_p, ctypes.c_longlong, c_double, c_double, c_void_p,
                                  c_void_p]),
    "gp_ode_dense": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_double, c_double,
                             ctypes.c_longlong, c_void_p, c_void_p]),
    "gp_ode_denoise": (c_int, [ctypes.POINTER(HeadWeights), c_void_p, c_float, c_float, c_float, c_float, c_void_p,
                               c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "gp_ode_ctl_size": (c_size_t, []),
    "gp_ode_auto_workspace_size": (c_size_t, [c_int]),
    "gp_ode_auto_attempt": (c_int, [ctypes.POINTER(HeadWeights), c_void_p, c_int, c_int, c_double, c_double, c_double,
                                    c_double, c_double, c_double, c_double, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_int, c_int, c_void_p, c_size_t, c_void_p]),
    "gp_ode_auto_attempt_hs": (c_int, [ctypes.POINTER(HeadWeights), c_void_p, c_int, c_int, c_double, c_double, c_double,
                                    c_double, c_double, c_double, c_double, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_int, c_int, c_void_p, c_size_t, c_void_p, c_void_p]),
    "gp_ode_global_partials": (c_int, [c_int, c_int, c_int, c_int]),
    "gp_ode_global_workspace_size": (c_size_t, [c_int]),
    "gp_ode_auto_partials_offset": (c_size_t, []),
    "gp_ode_auto_attempt_global": (c_int, [ctypes.POINTER(HeadWeights), c_void_p, c_int, c_int, c_double, c_double,
                                           c_double, c_double, c_double, c_double, c_double, c_void_p, c_void_p,
                                           c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                           c_int, c_int, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p,
                                           c_void_p]),
    "gp_pc_step_table": (c_int, [c_int, c_float, c_void_p]),
    "gp_ode_sample_workspace_size": (c_size_t, [c_int]),
    "gp_ode_sample": (c_int, [ctypes.POINTER(HeadWeights), c_void_p, c_void_p, c_int, c_int, c_double, c_double,
                              c_int, c_double, c_double, c_void_p, c_void_p, c_void_p, ctypes.POINTER(c_int),
                              ctypes.POINTER(c_int), c_void_p, c_size_t, c_void_p]),
    "gp_img_encoder_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "gp_img_encoder": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_float,
                               c_void_p, c_void_p, c_void_p, c_float, c_float, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_size_t, c_void_p]),
    "gp_img_encoder2": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_float,
                                c_void_p, c_void_p, c_void_p, c_float, c_float, c_void_p, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_void_p, c_size_t, c_void_p]),
    "gp_img_encoder3": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_float,
                                c_void_p, c_void_p, c_void_p, c_float, c_float, c_void_p, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_void_p, c_size_t, c_void_p]),
    "gp_img_encoder3_workspace_size": (c_size_t, [c_int, c_int, c_int, c_int]),
    "gp_img_geo_table": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p]),
    "gp_gather_patch_points": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int,
                                       c_void_p, c_void_p]),
    "gp_scale_forward": (c_int, [ctypes.POINTER(ScaleWeights), c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "gp_randn": (c_int, [c_uint64, ctypes.c_uint32, c_int, c_int, c_void_p, c_void_p]),
    "gp_points_mean": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "gp_bbox_length": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "gp_rank_aggregate": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float, c_int, c_void_p, c_void_p,
                                  c_void_p, c_void_p]),
}

EXPORTED = tuple(_SIGS)
_lib = None


# gp_pc_exchange_fn (genpose_hip.h): int (*)(void* ctx, int step, float* slot, int n, hipStream_t stream)
PC_EXCHANGE_FN = ctypes.CFUNCTYPE(c_int, c_void_p, c_int, c_void_p, c_int, c_void_p)
ODE_EXCHANGE_FN = PC_EXCHANGE_FN   # gp_ode_exchange_fn: the same C signature with an fp64 partials pointer


def load(path: str = LIB_PATH):
    """Load the HIP library (raises GenPoseHipError if it is absent or incomplete)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise GenPoseHipError(f"{path} not found: build it with `python -c 'import __graft_entry__ as g; "
                              f"g.build()'` (there is no CPU fallback)")
    lib = ctypes.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = load().gp_last_error().decode(errors="replace")
        raise GenPoseHipError(f"{what or 'genpose_hip'} failed ({rc}): {msg}")


def exported_symbols(path: str = LIB_PATH) -> Iterable[str]:
    lib = ctypes.CDLL(path)
    return [n for n in _SIGS if hasattr(lib, n)]
