"""ctypes binding of libmfnerf_hip.so (the C ABI declared in include/mfnerf.h).

This is the only way the Python host code reaches the GPU kernels.  There is no CPU
fallback: if the shared library is missing or fails to load, importing any op module
raises immediately (build it with `make -C mf-nerf_amd/csrc` or __graft_entry__.build()).
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MFNERF_LIB", os.path.join(os.path.dirname(_HERE), "libmfnerf_hip.so"))

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I = ctypes.c_int
_F = ctypes.c_float

MAX_LEVELS = 32


class GridDesc(ctypes.Structure):
    """mfnerf_grid_desc (include/mfnerf.h)."""
    _fields_ = [
        ("n_levels", ctypes.c_int32),
        ("n_features", ctypes.c_int32),
        ("canon_res", ctypes.c_int32),
        ("pad_", ctypes.c_int32),
        ("scale", ctypes.c_float * MAX_LEVELS),
        ("res", ctypes.c_uint32 * MAX_LEVELS),
        ("offset", ctypes.c_uint32 * MAX_LEVELS),
        ("size", ctypes.c_uint32 * MAX_LEVELS),
        ("table_kind", ctypes.c_int32 * MAX_LEVELS),
    ]


class AdamFused(ctypes.Structure):
    """mfnerf_adam_fused (include/mfnerf.h)."""
    _fields_ = [
        ("params", ctypes.c_void_p), ("m", ctypes.c_void_p), ("v", ctypes.c_void_p), ("p16", ctypes.c_void_p),
        ("table_offset", ctypes.c_int64),
        ("lr", ctypes.c_float), ("beta1", ctypes.c_float), ("beta2", ctypes.c_float), ("eps", ctypes.c_float),
        ("step_dev", ctypes.c_void_p), ("lr_dev", ctypes.c_void_p), ("amp", ctypes.c_void_p),
    ]


# name -> (restype, argtypes); mirrors include/mfnerf.h one to one
SIGNATURES = {
    "mfnerf_last_error": (ctypes.c_char_p, []),
    "mfnerf_abi_version": (_I, []),
    "mfnerf_ray_aabb_intersect": (_I, [_P, _P, _P, _P, _I64, _I64, _I, _P, _P, _P, _P]),
    "mfnerf_morton3d": (_I, [_P, _I64, _P, _P]),
    "mfnerf_morton3d_invert": (_I, [_P, _I64, _P, _P]),
    "mfnerf_packbits": (_I, [_P, _I64, _F, _P, _P, _P]),
    "mfnerf_raymarching_train_workspace": (_I64, [_I64, _I]),
    "mfnerf_raymarching_train": (_I, [_P, _P, _P, _I64, _P, _I, _F, _F, _P, _I, _I, _I64, _I64,
                                      _P, _P, _P, _P, _P, _P, _P, _P]),
    "mfnerf_raymarching_test": (_I, [_P, _P, _P, _I64, _P, _I64, _P, _I, _F, _F, _I, _I, _I,
                                     _P, _P, _P, _P, _P, _P]),
    "mfnerf_composite_train_fw": (_I, [_P, _P, _P, _P, _P, _I64, _I64, _F, _P, _P, _P, _P, _P, _P]),
    "mfnerf_composite_train_bw": (_I, [_P] * 13 + [_I64, _I64, _F, _P, _P, _P]),
    "mfnerf_composite_train_fused": (_I, [_P, _P, _P, _P, _P, _I64, _I64, _F, _P, _I64, _F, _F, _F, _F]
                                     + [_P] * 10 + [_P]),
    "mfnerf_composite_test_fw": (_I, [_P, _P, _P, _P, _P, _I64, _I, _F, _P, _P, _P, _P, _P]),
    "mfnerf_distortion_loss_fw": (_I, [_P, _P, _P, _P, _I64, _I64, _P, _P, _P, _P]),
    "mfnerf_distortion_loss_bw": (_I, [_P, _P, _P, _P, _P, _P, _P, _I64, _I64, _P, _P]),
    "mfnerf_nerf_loss": (_I, [_P, _P, _P, _I64, _I64, _F, _F, _F, _F, _P, _P, _P, _P]),
    "mfnerf_grid_encode_fw": (_I, [_P, _I64, _P, _F, _F, ctypes.POINTER(GridDesc), _P, _P, _P]),
    "mfnerf_grid_encode_fw_planar": (_I, [_P, _I64, _P, _F, _F, ctypes.POINTER(GridDesc), _P, _P, _I64, _P]),
    "mfnerf_grid_encode_bw_workspace": (_I64, [ctypes.POINTER(GridDesc)]),
    "mfnerf_grid_encode_bw": (_I, [_P, _I64, _P, _F, _F, ctypes.POINTER(GridDesc), _P, _P, _P, _P, _P]),
    "mfnerf_grid_encode_bw_scatter": (_I, [_P, _I64, _P, _F, _F, ctypes.POINTER(GridDesc), _P, _P, _P, _P, _P]),
    "mfnerf_grid_encode_bw_finish": (_I, [ctypes.POINTER(GridDesc), _P, _P, _P, _P]),
    "mfnerf_grid_encode_bw_binned_workspace": (_I64, [ctypes.POINTER(GridDesc), _I64]),
    "mfnerf_grid_encode_bw_binned": (_I, [_P, _I64, _P, _F, _F, ctypes.POINTER(GridDesc), _P, _P, _P, _I64, _P, _I,
                                          _P]),
    "mfnerf_grid_encode_bw_binned_float": (_I, [_P, _I64, _P, _F, _F, ctypes.POINTER(GridDesc), _P, _P, _P, _I64,
                                               _P, _P, _P, _I64, _I64, _I64, _P]),
    "mfnerf_grid_encode_bw_binned_adam": (_I, [_P, _I64, _P, _F, _F, ctypes.POINTER(GridDesc), _P, _P, _P, _I64,
                                              _P, ctypes.POINTER(AdamFused), _P]),
    "mfnerf_grid_encode_bw_binned_adam_all": (_I, [_P, _I64, _P, _F, _F, ctypes.POINTER(GridDesc), _P, _P, _I64, _P,
                                                  _I64, _P, ctypes.POINTER(AdamFused), _P, _P, _P, _I, _P, _P]),
    "mfnerf_grid_binned_first_value": (_I64, [ctypes.POINTER(GridDesc)]),
    "mfnerf_grid_dense_values": (_I64, [ctypes.POINTER(GridDesc)]),
    "mfnerf_grid_encode_bw_binned_flag_offset": (_I64, [ctypes.POINTER(GridDesc), _I64]),
    "mfnerf_grid_level_l1": (_I, [_P, _I64, _P, _I, _P, _P]),
    "mfnerf_field_packed_bytes": (_I64, [_I]),
    "mfnerf_field_pack_weights_f16": (_I, [_P, _P, _I, _P, _P]),
    "mfnerf_sh4_fw": (_I, [_P, _I64, _P, _P]),
    "mfnerf_field_pack_weights": (_I, [_P, _P, _I, _P, _P]),
    "mfnerf_field_fw": (_I, [_P, _I64, _P, _I64, _P, _P, _I, _I, _P, _P, _P]),
    "mfnerf_field_fw_density_scatter": (_I, [_P, _I64, _I64, _P, _P, _I, _P, _P, _P, _P]),
    "mfnerf_field_bw_workspace": (_I64, [_I64, _I]),
    "mfnerf_field_bw_slab_rows": (_I, [_I]),
    "mfnerf_field_bw": (_I, [_P, _I64, _P, _I64, _P, _P, _I, _P, _P, _F, _P, _P, _P, _P, _P, _P, _P]),
    "mfnerf_occupancy_workspace": (_I64, [_I, _I]),
    "mfnerf_occupancy_points": (_I64, [_I, _I, _I64, _I]),
    "mfnerf_occupancy_cells": (_I, [_P, _I, _I, _F, _I64, _I, _F, ctypes.c_uint64, ctypes.c_uint64, _P, _P, _P, _P]),
    "mfnerf_occupancy_cells_dev": (_I, [_P, _I, _I, _F, _I64, _I, _F, ctypes.c_uint64, _P, _P, _P, _P, _P]),
    "mfnerf_occupancy_update": (_I, [_P, _P, _P, _I64, _I, _I, _F, _P, _F, _P, _P, _P, _P]),
    "mfnerf_occupancy_points_unique": (_I64, [_I, _I, _I64, _I]),
    "mfnerf_occupancy_cells_unique": (_I, [_P, _I, _I, _F, _I64, _I, _F, ctypes.c_uint64, ctypes.c_uint64, _P, _P, _P,
                                           _P, _P]),
    "mfnerf_occupancy_cells_unique_dev": (_I, [_P, _I, _I, _F, _I64, _I, _F, ctypes.c_uint64, _P, _P, _P, _P, _P, _P]),
    "mfnerf_occupancy_update_dev": (_I, [_P, _P, _P, _I64, _P, _I, _I, _F, _P, _F, _P, _I, _P, _P, _P]),
    "mfnerf_sample_rays": (_I, [_P, _P, _P, _I64, _I64, _I64, _I, ctypes.c_uint64, _P, _P, _P, _P, _P]),
    "mfnerf_sample_rays_prep": (_I, [_P, _P, _P, _I64, _I64, _I64, _I, ctypes.c_uint64, _P, _P, _P, _P, _F, _P, _P,
                                     _P]),
    "mfnerf_adam_step": (_I, [_P, _P, _P, _P, _P, _I64, _F, _F, _F, _F, _F, _I, _P, _P, _P, _I, _P]),
    "mfnerf_adam_step_shard": (_I, [_P, _P, _P, _P, _P, _I64, _F, _F, _F, _F, _F, _P, _P, _P, _P, _I, _P]),
    "mfnerf_adam_step_fixed": (_I, [_P, _P, _P, _P, _P, _I64, _I64, ctypes.POINTER(GridDesc), _P, _P, _F, _F, _F, _F, _P, _P, _P, _P]),
    "mfnerf_adam_step_fixed_partial": (_I, [_P, _P, _P, _P, _P, _I64, _I64, ctypes.POINTER(GridDesc), _P, _P, _F, _F, _F,
                                            _F, _P, _P, _P, _I64, _P, _P]),
    "mfnerf_field_bw_reduce": (_I, [_I, _P, _P, _P, _P, _P]),
    "mfnerf_field_bw_reduce_store": (_I, [_I, _P, _P, _P, _P, _P]),
    "mfnerf_mlp_n_params": (_I64, [_I, _I, _I, _I]),
    "mfnerf_mlp_packed_bytes": (_I64, [_I, _I, _I, _I]),
    "mfnerf_mlp_pack": (_I, [_P, _I, _I, _I, _I, _P, _P]),
    "mfnerf_mlp_fw": (_I, [_P, _I64, _P, _I, _I, _I, _I, _I, _P, _P]),
    "mfnerf_mlp_bw_workspace": (_I64, [_I64, _I, _I, _I, _I]),
    "mfnerf_mlp_bw": (_I, [_P, _I64, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P]),
    "mfnerf_check_finite": (_I, [_P, _I64, _P, _P]),
    "mfnerf_flag_to_shards": (_I, [_P, _I64, _I64, _P, _P]),
    "mfnerf_flag_from_shard": (_I, [_P, _P, _P]),
    "mfnerf_gate_signal": (_I, [_P, _P]),
    "mfnerf_gate_wait": (_I, [_P, _I64, _P]),
}

_lib = None


def load():
    """Load and type the library once; raises if it is absent (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libmfnerf_hip.so not found at {LIB_PATH}: build it with "
                          f"`make -C mf-nerf_amd/csrc` (or __graft_entry__.build())")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def call(name, *args):
    """Call an entry point; a nonzero status becomes RuntimeError (binding.cpp CHECK_* -> c10::Error)."""
    st = getattr(load(), name)(*args)
    if st != 0:
        msg = load().mfnerf_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed ({st}): {msg}")


def ptr(t):
    """Device pointer of a tensor for the C ABI (None -> NULL).  Host tensors are refused: every
    pointer this library takes is dereferenced on the GPU."""
    if t is None:
        return ctypes.c_void_p(0)
    if not t.is_cuda:
        raise ValueError("libmfnerf_hip takes device tensors; got a host tensor")
    return ctypes.c_void_p(t.data_ptr())


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def check_input(name, t, dtype=None):
    """CHECK_INPUT of models/csrc/include/utils.h:4-6 plus the implicit accessor dtype check."""
    if not isinstance(t, torch.Tensor):
        raise RuntimeError(f"{name} must be a tensor")
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA tensor")
    if not t.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous")
    if dtype is not None and t.dtype != dtype:
        raise RuntimeError(f"{name} must be {dtype}, got {t.dtype}")
