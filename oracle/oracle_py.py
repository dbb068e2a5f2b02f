"""ctypes binding of the CPU oracle (oracle/liboracle.so) and of oracle/_ref.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg — never by the product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"
REF_LIB = HERE / "_ref" / "libref_ply.so"
POINT_FLOATS = 62

RECORD_DTYPE = np.dtype([("cx", "<f4"), ("cy", "<f4"), ("ax", "<f4"), ("ay", "<f4"), ("bx", "<f4"),
                         ("by", "<f4"), ("opacity", "<f4"), ("r", "<f4"), ("g", "<f4"), ("b", "<f4"),
                         ("rect_lo", "<u4"), ("rect_hi", "<u4")])


class OraScene(C.Structure):
    _fields_ = [("n", C.c_int64), ("pos", C.c_void_p), ("rot", C.c_void_p), ("scale", C.c_void_p),
                ("opacity", C.c_void_p), ("color", C.c_void_p), ("sh_rest", C.c_void_p), ("sh_degree", C.c_int)]


class OraDebug(C.Structure):
    _fields_ = [("zf", C.c_float), ("a", C.c_float), ("b", C.c_float), ("c", C.c_float), ("r1", C.c_float),
                ("r2", C.c_float), ("e1x", C.c_float), ("e1y", C.c_float), ("dkey", C.c_uint32),
                ("ntiles", C.c_uint32), ("visible", C.c_int)]


class OraOptions(C.Structure):
    _fields_ = [("mode", C.c_int), ("cap", C.c_int), ("nthreads", C.c_int)]


class OraStats(C.Structure):
    _fields_ = [("visible", C.c_int64), ("pairs", C.c_int64), ("tiles", C.c_int64)]


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB.exists():
            subprocess.run(["make", "-s", "-C", str(HERE), "liboracle.so"], check=True)
        L = C.CDLL(str(LIB))
        L.ora_ply_load.argtypes = [C.c_char_p, C.POINTER(C.POINTER(C.c_float)), C.POINTER(C.c_int64)]
        L.ora_ply_load.restype = C.c_int
        L.ora_free.argtypes = [C.c_void_p]
        L.ora_crop.argtypes = [C.c_void_p, C.c_int64, C.c_float, C.c_void_p]
        L.ora_crop.restype = C.c_int64
        L.ora_look_at.argtypes = [C.c_void_p] * 4
        L.ora_perspective.argtypes = [C.c_float] * 4 + [C.c_void_p]
        L.ora_mat4_mul.argtypes = [C.c_void_p] * 3
        L.ora_camera_position.argtypes = [C.c_void_p] * 2
        L.ora_project.argtypes = [C.POINTER(OraScene), C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                  C.c_int, C.c_int, C.c_void_p, C.POINTER(OraDebug)]
        L.ora_project_all.argtypes = [C.POINTER(OraScene), C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p,
                                      C.c_void_p, C.c_void_p, C.c_int]
        L.ora_render.argtypes = [C.POINTER(OraScene), C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                                 C.POINTER(OraOptions), C.c_void_p, C.POINTER(OraStats)]
        L.ora_render.restype = C.c_int
        L.ora_composite_records.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_int,
                                            C.POINTER(OraOptions), C.c_void_p, C.c_int, C.c_int, C.c_void_p,
                                            C.POINTER(OraStats)]
        L.ora_composite_records.restype = C.c_int
        L.ora_composite_slab.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_int, C.POINTER(OraOptions),
                                         C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        L.ora_composite_slab.restype = C.c_int
        L.ora_composite_list.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]
        L.ora_f32_to_f16_bits.argtypes = [C.c_float]
        L.ora_f32_to_f16_bits.restype = C.c_uint16
        L.ora_expf.argtypes = [C.c_float]
        L.ora_expf.restype = C.c_float
        L.ora_gauss.argtypes = [C.c_float]
        L.ora_gauss.restype = C.c_float
        L.ora_gauss2.argtypes = [C.c_float]
        L.ora_gauss2.restype = C.c_float
        L.ora_to_bgra8.argtypes = [C.c_void_p, C.c_int64, C.c_void_p]
        L.ora_to_bgra8.restype = None
        _lib = L
    return _lib


_MODES = {"tile": 0, "live50": 1, "mlab": 2}  # ORA_MODE_*


def _col16(m) -> np.ndarray:
    a = np.asarray(m, np.float32)
    if a.shape == (4, 4):
        a = a.T
    return np.ascontiguousarray(a.reshape(16), np.float32)


def _scene(scene, sh_degree: int):
    keep = [np.ascontiguousarray(getattr(scene, f), np.float32) if getattr(scene, f) is not None else None
            for f in ("pos", "rot", "scale", "opacity", "color", "sh_rest")]
    s = OraScene()
    s.n = keep[0].shape[0]
    s.pos, s.rot, s.scale, s.opacity, s.color = (k.ctypes.data for k in keep[:5])
    s.sh_rest = keep[5].ctypes.data if keep[5] is not None else None
    s.sh_degree = int(sh_degree)
    return s, keep


def ply_load(path) -> tuple[bool, np.ndarray]:
    ptr = C.POINTER(C.c_float)()
    n = C.c_int64(0)
    ok = lib().ora_ply_load(str(path).encode(), C.byref(ptr), C.byref(n))
    pts = np.zeros((0, POINT_FLOATS), np.float32)
    if n.value > 0:
        pts = np.ctypeslib.as_array(ptr, shape=(n.value * POINT_FLOATS,)).reshape(-1, POINT_FLOATS).copy()
    if ptr:
        lib().ora_free(ptr)
    return bool(ok), pts


def crop(points: np.ndarray, radius: float = 5.0) -> np.ndarray:
    p = np.ascontiguousarray(points, np.float32)
    keep = np.zeros(p.shape[0], np.int64)
    k = lib().ora_crop(p.ctypes.data, p.shape[0], float(radius), keep.ctypes.data)
    return keep[:k]


def look_at(eye, center, up) -> np.ndarray:
    out = np.zeros(16, np.float32)
    a = [np.asarray(v, np.float32) for v in (eye, center, up)]
    lib().ora_look_at(a[0].ctypes.data, a[1].ctypes.data, a[2].ctypes.data, out.ctypes.data)
    return out.reshape(4, 4).T.copy()


def perspective(fov_deg, aspect, zn, zf) -> np.ndarray:
    out = np.zeros(16, np.float32)
    lib().ora_perspective(float(fov_deg), float(aspect), float(zn), float(zf), out.ctypes.data)
    return out.reshape(4, 4).T.copy()


def mat4_mul(a, b) -> np.ndarray:
    out = np.zeros(16, np.float32)
    A, B = _col16(a), _col16(b)
    lib().ora_mat4_mul(A.ctypes.data, B.ctypes.data, out.ctypes.data)
    return out.reshape(4, 4).T.copy()


def project(scene, view, proj, width, height, sh_degree=0, nthreads=0):
    s, keep = _scene(scene, sh_degree)
    n = s.n
    rec = np.zeros(n, RECORD_DTYPE)
    dk = np.zeros(n, np.uint32)
    nt = np.zeros(n, np.uint32)
    V, P = _col16(view), _col16(proj)
    lib().ora_project_all(C.byref(s), V.ctypes.data, P.ctypes.data, int(width), int(height), rec.ctypes.data,
                          dk.ctypes.data, nt.ctypes.data, int(nthreads))
    return rec, dk, nt


def project_debug(scene, view, proj, width, height, sh_degree=0):
    """Per-splat K1-K5 intermediates (ora_project): records and a dict of
    arrays zf, a, b, c, r1, r2, e1x, e1y, dkey, ntiles, visible."""
    s, keep = _scene(scene, sh_degree)
    V, P = _col16(view), _col16(proj)
    VP = np.zeros(16, np.float32)
    cam = np.zeros(3, np.float32)
    lib().ora_mat4_mul(P.ctypes.data, V.ctypes.data, VP.ctypes.data)
    lib().ora_camera_position(V.ctypes.data, cam.ctypes.data)
    rec = np.zeros(s.n, RECORD_DTYPE)
    dbg = {k: np.zeros(s.n, np.float32 if t is C.c_float else np.int64) for k, t in OraDebug._fields_}
    d = OraDebug()
    for i in range(s.n):
        lib().ora_project(C.byref(s), i, V.ctypes.data, P.ctypes.data, VP.ctypes.data, cam.ctypes.data, int(width),
                          int(height), rec[i:i + 1].ctypes.data, C.byref(d))
        for k, _ in OraDebug._fields_:
            dbg[k][i] = getattr(d, k)
    return rec, dbg


def render(scene, view, proj, width, height, sh_degree=0, mode="tile", cap=0, nthreads=0):
    s, keep = _scene(scene, sh_degree)
    out = np.zeros((height, width, 4), np.float32)
    o = OraOptions(_MODES[mode], int(cap), int(nthreads))
    st = OraStats()
    V, P = _col16(view), _col16(proj)
    lib().ora_render(C.byref(s), V.ctypes.data, P.ctypes.data, int(width), int(height), C.byref(o),
                     out.ctypes.data, C.byref(st))
    return out, {"visible": st.visible, "pairs": st.pairs, "tiles": st.tiles}


def composite_records(rec, dkey, width, height, owner=None, rank=0, compact=False, mode="tile", cap=0,
                      nthreads=0):
    """Bin/sort/composite an explicit record list (index = arrival order).
    owner: uint8 per 32-px row (None = all rows owned)."""
    rec = np.ascontiguousarray(rec, RECORD_DTYPE)
    dkey = np.ascontiguousarray(dkey, np.uint32)
    own = None if owner is None else np.ascontiguousarray(owner, np.uint8)
    rows = int((own == rank).sum()) * 32 if (compact and own is not None) else height
    out = np.zeros((rows, width, 4), np.float32)
    o = OraOptions(_MODES[mode], int(cap), int(nthreads))
    st = OraStats()
    lib().ora_composite_records(rec.ctypes.data, dkey.ctypes.data, rec.shape[0], int(width), int(height),
                                C.byref(o), None if own is None else own.ctypes.data, int(rank),
                                int(bool(compact)), out.ctypes.data, C.byref(st))
    return out


def composite_slab(rec, dkey, width, height, pas, rank=0, t_all=None, mode="tile", nthreads=0):
    """Depth-slab passes (gs_oracle.h ora_composite_slab): pass 1 -> (H, W)
    transmittance, pass 2 -> (H, W, 4) contributions from t_all [world, H, W]."""
    rec = np.ascontiguousarray(rec, RECORD_DTYPE)
    dkey = np.ascontiguousarray(dkey, np.uint32)
    out = np.zeros((height, width) if pas == 1 else (height, width, 4), np.float32)
    ta = None if t_all is None else np.ascontiguousarray(t_all, np.float32)
    o = OraOptions(_MODES[mode], 0, int(nthreads))
    ok = lib().ora_composite_slab(rec.ctypes.data, dkey.ctypes.data, rec.shape[0], int(width), int(height),
                                  C.byref(o), int(pas), int(rank), None if ta is None else ta.ctypes.data,
                                  out.ctypes.data)
    if not ok:
        raise ValueError("ora_composite_slab: bad arguments")
    return out


def composite_list(frags, mode="tile", cap=0) -> np.ndarray:
    f = np.ascontiguousarray(frags, np.float32).reshape(-1, 5)
    out = np.zeros(4, np.float32)
    lib().ora_composite_list(f.ctypes.data, f.shape[0], _MODES[mode], int(cap), out.ctypes.data)
    return out


def f16_bits(x: float) -> int:
    return int(lib().ora_f32_to_f16_bits(float(x)))


def expf(x: float) -> float:
    return float(lib().ora_expf(float(x)))


def gauss(q: float) -> float:
    return float(lib().ora_gauss(float(q)))


def gauss2(qs: float) -> float:
    """2^-qs, the composite's gaussian on the scaled conic."""
    return float(lib().ora_gauss2(float(qs)))


def to_bgra8(rgba: np.ndarray) -> np.ndarray:
    """(H, W, 4) fp32 RGBA -> (H, W, 4) uint8 BGRA8Unorm."""
    f = np.ascontiguousarray(rgba, dtype=np.float32)
    out = np.empty(f.shape[:-1] + (4,), np.uint8)
    lib().ora_to_bgra8(f.ctypes.data, f.size // 4, out.ctypes.data)
    return out


# ---- oracle/_ref: the reference's own loader, compiled from /root/reference ----
_ref = None


def ref_available() -> bool:
    return REF_LIB.exists()


def ref_ply_load(path) -> tuple[bool, np.ndarray]:
    global _ref
    if _ref is None:
        _ref = C.CDLL(str(REF_LIB))
        _ref.ref_ply_load.argtypes = [C.c_char_p, C.c_void_p, C.c_longlong]
        _ref.ref_ply_load.restype = C.c_longlong
    n = _ref.ref_ply_load(str(path).encode(), None, 0)
    ok = n >= 0
    cnt = n if ok else -1 - n
    out = np.zeros((max(cnt, 0), POINT_FLOATS), np.float32)
    if cnt > 0:
        _ref.ref_ply_load(str(path).encode(), out.ctypes.data, cnt)
    return ok, out
