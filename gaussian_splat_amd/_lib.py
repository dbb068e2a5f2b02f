"""ctypes binding of libgsplat.so (the C-ABI declared in include/gsplat.h).

The product path has exactly one implementation: the HIP kernels inside
libgsplat.so.  If the library is missing this module raises — there is no CPU
fallback anywhere in the package.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

# GSPLAT_LIB: development aid to A/B a differently built libgsplat (tools/ab.sh)
LIB_PATH = Path(os.environ.get("GSPLAT_LIB") or Path(__file__).resolve().parent / "libgsplat.so")


class GsOptions(C.Structure):
    _fields_ = [("mode", C.c_int32), ("sh_degree", C.c_int32), ("crop", C.c_int32),
                ("crop_radius", C.c_float), ("stage_timing", C.c_int32), ("cap", C.c_int32),
                ("frames_in_flight", C.c_int32),
                ("binning", C.c_int32), ("depth_split", C.c_int32),
                ("reserved", C.c_int32 * 3)]


class GsSceneSoa(C.Structure):
    _fields_ = [("n", C.c_int64), ("pos", C.c_void_p), ("rot", C.c_void_p), ("scale", C.c_void_p),
                ("opacity", C.c_void_p), ("color", C.c_void_p), ("sh_rest", C.c_void_p)]


class GsStats(C.Structure):
    _fields_ = [("splats", C.c_int64), ("visible", C.c_int64), ("pairs", C.c_int64), ("tiles", C.c_int64),
                ("width", C.c_int32), ("height", C.c_int32), ("sort_bits", C.c_int32), ("sort_passes", C.c_int32),
                ("ms_preprocess", C.c_float), ("ms_scan", C.c_float), ("ms_duplicate", C.c_float),
                ("ms_sort", C.c_float), ("ms_ranges", C.c_float), ("ms_composite", C.c_float),
                ("ms_total", C.c_float),
                ("bytes_preprocess", C.c_int64), ("bytes_scan", C.c_int64), ("bytes_duplicate", C.c_int64),
                ("bytes_sort", C.c_int64), ("bytes_ranges", C.c_int64), ("bytes_composite", C.c_int64),
                ("ms_depth_sort", C.c_float), ("ms_exchange", C.c_float), ("bytes_depth_sort", C.c_int64),
                ("binning", C.c_int32), ("front_only", C.c_int32), ("records_fetched", C.c_int64),
                ("pairs_sorted", C.c_int64), ("open_tiles", C.c_int64), ("cut_frame", C.c_int32),
                ("cut_dilate", C.c_uint32)]

    def as_dict(self) -> dict:
        d = {k: getattr(self, k) for k, _ in self._fields_}
        # deprecated aliases of the ABI-10 renames (gsplat.h gs_stats), kept for one release
        d["two_slab"], d["depth_cut"] = d["cut_frame"], d["cut_dilate"]
        return d


# name -> (restype, argtypes); every symbol include/gsplat.h declares.
_P = C.c_void_p
_FP = C.POINTER(C.c_float)
_I64P = C.POINTER(C.c_int64)
SIGNATURES = {
    "gs_abi_version": (C.c_int32, []),
    "gs_last_error": (C.c_char_p, []),
    "gs_default_options": (None, [C.POINTER(GsOptions)]),
    "gs_create": (C.c_int, [C.c_char_p, C.POINTER(GsOptions), C.POINTER(_P)]),
    "gs_create_from_soa": (C.c_int, [C.POINTER(GsSceneSoa), C.POINTER(GsOptions), C.POINTER(_P)]),
    "gs_create_from_points": (C.c_int, [_P, C.c_int64, C.POINTER(GsOptions), C.POINTER(_P)]),
    "gs_create_subset": (C.c_int, [_P, C.c_int64, C.c_int64, C.POINTER(_P)]),
    "gs_get_scene": (C.c_int, [_P, _P, _P, _P, _P, _P, _P]),
    "gs_initialize": (C.c_int, [_P, C.c_int32]),
    "gs_point_count": (C.c_int64, [_P]),
    "gs_destroy": (None, [_P]),
    "gs_set_mode": (C.c_int, [_P, C.c_int32]),
    "gs_set_cap": (C.c_int, [_P, C.c_int32]),
    "gs_set_depth_split": (C.c_int, [_P, C.c_int32]),
    "gs_set_stage_timing": (C.c_int, [_P, C.c_int32]),
    "gs_set_frames_in_flight": (C.c_int, [_P, C.c_int32]),
    "gs_render": (C.c_int, [_P, _FP, _FP, C.c_int32, C.c_int32, _P, C.c_int32, _P]),
    "gs_render_bgra8": (C.c_int, [_P, _FP, _FP, C.c_int32, C.c_int32, _P, C.c_int32, _P]),
    "gs_last_stats": (C.c_int, [_P, C.POINTER(GsStats)]),
    "gs_kernel_times": (C.c_int, [_P, C.c_int32, _FP, _FP, C.POINTER(C.c_int32)]),
    "gs_project_host": (C.c_int, [_P, _FP, _FP, C.c_int32, C.c_int32, _P, _P, _P]),
    "gs_sorted_pairs_host": (C.c_int, [_P, _P, _P, C.c_int64, _I64P]),
    "gs_radix_sort_pairs": (C.c_int, [_P, _P, _P, _P, C.c_int64, C.c_int32, _P]),
    "gs_shard_configure": (C.c_int, [_P, C.c_int32, C.c_int32, C.c_int64]),
    "gs_shard_set_rows": (C.c_int, [_P, _P, C.c_int32]),
    "gs_shard_project": (C.c_int, [_P, _FP, _FP, C.c_int32, C.c_int32, _P, C.c_int64, _I64P, _P]),
    "gs_shard_render": (C.c_int, [_P, _P, C.c_int64, C.c_int32, C.c_int32, _P, _P]),
    "gs_shard_render_split": (C.c_int, [_P, _P, C.c_int64, C.c_int32, C.c_int32, _P, _P, _P]),
    "gs_band_render": (C.c_int, [_P, _FP, _FP, C.c_int32, C.c_int32, _P, _P]),
    "gs_exchange_record_bytes": (C.c_int32, []),
    "gs_exchange_regions": (C.c_int32, [C.c_void_p]),
    "gs_slab_project": (C.c_int, [_P, _FP, _FP, C.c_int32, C.c_int32, _P, _P]),
    "gs_slab_bounds": (C.c_int, [_P, C.c_int32, _P]),
    "gs_slab_pack": (C.c_int, [_P, _P, _P, C.c_int64, _I64P, _P]),
    "gs_slab_render": (C.c_int, [_P, _P, C.c_int64, C.c_int32, C.c_int32, _P, _P]),
    "gs_slab_composite": (C.c_int, [_P, _P, _P, _P]),
    "gs_create_sharded": (C.c_int, [C.c_char_p, C.POINTER(GsOptions), C.c_int32, C.POINTER(_P)]),
    "gs_create_sharded_from_handle": (C.c_int, [_P, C.c_int32, C.POINTER(_P)]),
    "gs_create_replicated": (C.c_int, [C.c_char_p, C.POINTER(GsOptions), C.c_int32, C.POINTER(_P)]),
    "gs_create_replicated_from_handle": (C.c_int, [_P, C.c_int32, C.POINTER(_P)]),
    "gs_group_initialize": (C.c_int, [_P, _P, C.c_int32]),
    "gs_group_set_scheme": (C.c_int, [_P, C.c_int32]),
    "gs_group_set_timeout": (C.c_int, [_P, C.c_int32]),
    "gs_group_render": (C.c_int, [_P, _FP, _FP, C.c_int32, C.c_int32, _P, C.c_int32, _P]),
    "gs_group_set_frames_in_flight": (C.c_int, [_P, C.c_int32]),
    "gs_group_render_pipelined": (C.c_int, [_P, _FP, _FP, C.c_int32, C.c_int32, _P, C.c_int32, _P,
                                            C.POINTER(C.c_int32)]),
    "gs_group_flush": (C.c_int, [_P, _P, C.c_int32, _P, C.POINTER(C.c_int32)]),
    "gs_group_point_count": (C.c_int64, [_P]),
    "gs_group_size": (C.c_int32, [_P]),
    "gs_group_transport": (C.c_int32, [_P]),
    "gs_group_last_stats": (C.c_int, [_P, C.c_int32, C.POINTER(GsStats)]),
    "gs_group_destroy": (None, [_P]),
    "gs_ply_load": (C.c_int, [C.c_char_p, C.c_int32, C.POINTER(_FP), _I64P]),
    "gs_ply_free": (None, [_FP]),
    "gs_look_at": (None, [_FP, _FP, _FP, _FP]),
    "gs_perspective": (None, [C.c_float, C.c_float, C.c_float, C.c_float, _FP]),
}

STATUS = {0: "GS_OK", 1: "GS_ERR_INVALID_ARG", 2: "GS_ERR_IO", 3: "GS_ERR_PARSE", 4: "GS_ERR_DEVICE",
          5: "GS_ERR_OOM", 6: "GS_ERR_COMM", 7: "GS_ERR_UNSUPPORTED", 8: "GS_ERR_STATE"}


class GsError(RuntimeError):
    def __init__(self, status: int, what: str):
        self.status = status
        super().__init__(f"{what}: {STATUS.get(status, status)}: {last_error()}")


_lib: C.CDLL | None = None


def lib() -> C.CDLL:
    """Load libgsplat.so; raises if it was not built (no fallback)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise ImportError(f"{LIB_PATH} is missing: run `python -m gaussian_splat_amd.build` "
                              "(the HIP extension is required; there is no CPU path)")
        L = C.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def last_error() -> str:
    if _lib is None:
        return ""
    v = _lib.gs_last_error()
    return v.decode() if v else ""


def check(status: int, what: str) -> None:
    if status != 0:
        raise GsError(status, what)
