"""Python mirror of the reference's host API over libgsplat.so.

Names follow the reference (nshelton/gaussian_splat):
  InstancedSplatRenderer  src/instanced_splat_renderer.h:13-34
  PLYLoader.load          src/ply_loader.h:30-44
  TrackballCamera         src/trackball_camera.h:5-64
with the Metal command buffer / drawable replaced by a HIP stream and an HBM
framebuffer (a torch CUDA tensor of shape (H, W, 4), fp32 RGBA, y down).

Matrices are 4x4 numpy arrays in math convention (M[row, col]); they cross
the C-ABI column-major, exactly like simd_float4x4.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _lib as L
from ._lib import GsOptions, GsSceneSoa, GsStats, check, lib

POINT_FLOATS = 62  # sizeof(PointData) / 4, src/ply_loader.h:7-28
RECORD_DTYPE = np.dtype([("cx", "<f4"), ("cy", "<f4"), ("ax", "<f4"), ("ay", "<f4"), ("bx", "<f4"),
                         ("by", "<f4"), ("opacity", "<f4"), ("r", "<f4"), ("g", "<f4"), ("b", "<f4"),
                         ("rect_lo", "<u4"), ("rect_hi", "<u4")])
MODES = {"tile": 0, "live50": 1, "mlab": 2}
BINNING = {"default": 0, "depth_first": 1, "bin_first": 2}  # gs_binning


def _mat16(m) -> C.Array:
    a = np.asarray(m, dtype=np.float32)
    if a.shape == (4, 4):
        a = a.T  # math convention -> column-major
    a = np.ascontiguousarray(a.reshape(16), dtype=np.float32)
    return (C.c_float * 16)(*a.tolist())


def _from16(buf) -> np.ndarray:
    return np.array(list(buf), dtype=np.float32).reshape(4, 4).T.copy()


@dataclass
class Options:
    mode: str = "tile"
    sh_degree: int = 0
    crop: bool = True
    crop_radius: float = 5.0
    stage_timing: int = 0  # 0 off, 1 every stage (adds event gaps), 2 preprocess + composite only
    cap: int = 0  # per-pixel fragment cap by arrival order (0 = none; 32 tile shader, 50 live shader)
    frames_in_flight: int = 1  # 2: projection/sort of a frame overlaps the previous frame's composite
    # bin-list build order: "default" (per frame from the previous frame's pair count at this
    # resolution; depth-first on the first frame), "depth_first", "bin_first"
    binning: str = "default"
    # per-bin depth cuts (gs_options.depth_split; tile/live50 rules, no cap): a frame's
    # bin lists hold the pairs in front of the depth at which the bin's tiles saturated two frames
    # back, and a quadrant those lists leave open finishes from its saved state with the rest of
    # its bin's pairs.  Single-GPU frames, row-scheme rank renders and contiguous band renders alike.
    # The same image bit for bit, fewer pairs sorted; True is the default (False: whole lists)
    depth_split: bool = True

    def to_c(self) -> GsOptions:
        o = GsOptions()
        lib().gs_default_options(C.byref(o))
        if self.mode not in MODES:
            raise ValueError(f"mode must be one of {list(MODES)}")
        o.mode = MODES[self.mode]
        o.sh_degree = int(self.sh_degree)
        o.crop = int(bool(self.crop))
        o.crop_radius = float(self.crop_radius)
        o.stage_timing = int(self.stage_timing)
        if int(self.cap) < 0:
            raise ValueError("cap must be >= 0")
        o.cap = int(self.cap)
        if int(self.frames_in_flight) not in (1, 2):
            raise ValueError("frames_in_flight must be 1 or 2")
        o.frames_in_flight = int(self.frames_in_flight)
        if self.binning not in BINNING:
            raise ValueError(f"binning must be one of {list(BINNING)}")
        o.binning = BINNING[self.binning]
        o.depth_split = 1 if self.depth_split else 0
        return o


@dataclass
class Scene:
    """Host SoA scene (float32): activated values, as PLYLoader produces them."""
    pos: np.ndarray       # (N, 3)
    rot: np.ndarray       # (N, 4) w x y z raw
    scale: np.ndarray     # (N, 3) exp(scale)
    opacity: np.ndarray   # (N,) sigmoid(opacity)
    color: np.ndarray     # (N, 3) rgb (sh_degree 0) or raw f_dc (sh_degree > 0)
    sh_rest: Optional[np.ndarray] = None  # (N, 45) PLY order

    def __post_init__(self):
        for f in ("pos", "rot", "scale", "opacity", "color", "sh_rest"):
            v = getattr(self, f)
            if v is not None:
                setattr(self, f, np.ascontiguousarray(v, dtype=np.float32))

    @property
    def n(self) -> int:
        return int(self.pos.shape[0])

    @staticmethod
    def from_points(points: np.ndarray) -> "Scene":
        p = np.asarray(points, dtype=np.float32).reshape(-1, POINT_FLOATS)
        return Scene(pos=p[:, 0:3], rot=p[:, 13:17], scale=p[:, 10:13], opacity=p[:, 9], color=p[:, 6:9],
                     sh_rest=p[:, 17:62])

    def subset(self, sl) -> "Scene":
        return Scene(self.pos[sl], self.rot[sl], self.scale[sl], self.opacity[sl], self.color[sl],
                     None if self.sh_rest is None else self.sh_rest[sl])

    def to_c(self) -> GsSceneSoa:
        s = GsSceneSoa()
        s.n = self.n
        s.pos = self.pos.ctypes.data
        s.rot = self.rot.ctypes.data
        s.scale = self.scale.ctypes.data
        s.opacity = self.opacity.ctypes.data
        s.color = self.color.ctypes.data
        s.sh_rest = self.sh_rest.ctypes.data if self.sh_rest is not None else None
        return s


class PLYLoader:
    """src/ply_loader.h:30-44 — load() returns (ok, points[N, 62])."""

    @staticmethod
    def load(filepath: str, compat: bool = True) -> tuple[bool, np.ndarray]:
        ptr = L._FP()
        n = C.c_int64(0)
        st = lib().gs_ply_load(str(filepath).encode(), int(compat), C.byref(ptr), C.byref(n))
        pts = np.zeros((0, POINT_FLOATS), np.float32)
        if n.value > 0:
            pts = np.ctypeslib.as_array(ptr, shape=(n.value * POINT_FLOATS,)).reshape(-1, POINT_FLOATS).copy()
            lib().gs_ply_free(ptr)
        return st == 0, pts


def look_at(eye, center, up) -> np.ndarray:
    out = (C.c_float * 16)()
    f3 = lambda v: (C.c_float * 3)(*[float(x) for x in v])
    lib().gs_look_at(f3(eye), f3(center), f3(up), out)
    return _from16(out)


def perspective(fov_degrees: float, aspect: float, znear: float, zfar: float) -> np.ndarray:
    out = (C.c_float * 16)()
    lib().gs_perspective(float(fov_degrees), float(aspect), float(znear), float(zfar), out)
    return _from16(out)


class TrackballCamera:
    """src/trackball_camera.h:5-64 (matrix producers; defaults .mm:5-17, .h:28-37)."""

    def __init__(self):
        self.position = np.array([0.0, 0.0, 5.0], np.float32)
        self.target = np.zeros(3, np.float32)
        self.up = np.array([0.0, -1.0, 0.0], np.float32)
        self.distance = 5.0
        self.viewport = (800, 600)
        self.fov, self.nearPlane, self.farPlane = 45.0, 0.1, 1000.0
        self.minDistance, self.maxDistance = 0.1, 100.0

    def setViewportSize(self, w: int, h: int):
        self.viewport = (int(w), int(h))

    def setTarget(self, t):
        self.target = np.asarray(t, np.float32)

    def setPosition(self, p):
        self.position = np.asarray(p, np.float32)
        self.distance = float(np.linalg.norm(self.position - self.target))

    def setDistance(self, d: float):
        self.distance = min(max(d, self.minDistance), self.maxDistance)
        v = self.position - self.target
        self.position = self.target + v / np.linalg.norm(v) * self.distance

    def orbit(self, yaw: float, pitch: float = 0.0):
        """Rotate the eye about the target (trackball drag, .mm:55-83)."""
        off = self.position - self.target
        cy, sy = math.cos(yaw), math.sin(yaw)
        off = np.array([cy * off[0] + sy * off[2], off[1], -sy * off[0] + cy * off[2]], np.float32)
        if pitch:
            r = np.cross(-off, [0, 1, 0])
            r = r / np.linalg.norm(r)
            c, s = math.cos(pitch), math.sin(pitch)
            off = (off * c + np.cross(r, off) * s + r * np.dot(r, off) * (1 - c)).astype(np.float32)
        self.position = self.target + off

    def getViewMatrix(self) -> np.ndarray:
        return look_at(self.position, self.target, self.up)

    def getProjectionMatrix(self) -> np.ndarray:
        w, h = self.viewport
        return perspective(self.fov, np.float32(w) / np.float32(h), self.nearPlane, self.farPlane)


def default_camera(width: int, height: int) -> TrackballCamera:
    """The reference app's camera: eye (0,2,5), target 0 (src/main.mm:55-58)."""
    cam = TrackballCamera()
    cam.setViewportSize(width, height)
    cam.setPosition([0.0, 2.0, 5.0])
    cam.setTarget([0.0, 0.0, 0.0])
    return cam


class InstancedSplatRenderer:
    """src/instanced_splat_renderer.h:13-34 over libgsplat.so."""

    def __init__(self, source, options: Optional[Options] = None):
        self.options = options or Options()
        self._h = C.c_void_p()
        opt = self.options.to_c()
        if isinstance(source, Scene):
            self._scene_c = source.to_c()
            self._keep = source
            check(lib().gs_create_from_soa(C.byref(self._scene_c), C.byref(opt), C.byref(self._h)), "gs_create_from_soa")
        elif isinstance(source, np.ndarray):
            pts = np.ascontiguousarray(source, np.float32).reshape(-1, POINT_FLOATS)
            check(lib().gs_create_from_points(pts.ctypes.data, pts.shape[0], C.byref(opt), C.byref(self._h)),
                  "gs_create_from_points")
        else:
            check(lib().gs_create(str(source).encode(), C.byref(opt), C.byref(self._h)), "gs_create")
        self.device = None

    def initialize(self, device: int = 0) -> bool:
        check(lib().gs_initialize(self._h, int(device)), "gs_initialize")
        self.device = int(device)
        return True

    def getPointCount(self) -> int:
        return int(lib().gs_point_count(self._h))

    get_point_count = getPointCount

    def set_mode(self, mode: str):
        check(lib().gs_set_mode(self._h, MODES[mode]), "gs_set_mode")
        self.options.mode = mode

    def set_stage_timing(self, mode: int):
        """0 off, 1 every stage, 2 preprocess + composite via their own dispatch packets."""
        check(lib().gs_set_stage_timing(self._h, int(mode)), "gs_set_stage_timing")
        self.options.stage_timing = int(mode)

    def set_frames_in_flight(self, n: int):
        """1: every stage on the caller's stream; 2: a frame's projection/sort
        overlaps the previous frame's composite (internal stream)."""
        check(lib().gs_set_frames_in_flight(self._h, int(n)), "gs_set_frames_in_flight")
        self.options.frames_in_flight = int(n)

    def set_cap(self, cap: int):
        """Per-pixel fragment cap by arrival order (0 = none)."""
        check(lib().gs_set_cap(self._h, int(cap)), "gs_set_cap")
        self.options.cap = int(cap)

    def set_depth_split(self, on: bool):
        """Per-bin depth cuts (gs_set_depth_split): bin lists cut behind the depth
        where each bin saturated two frames back, open tiles finished by fallback
        lists; same image, bit for bit, less sorting."""
        check(lib().gs_set_depth_split(self._h, 1 if on else 0), "gs_set_depth_split")
        self.options.depth_split = bool(on)

    def render(self, view, proj, width: int, height: int, out=None, stream=None):
        """Render into `out` (torch float32 CUDA tensor (H, W, 4)); returns it."""
        import torch

        if out is None:
            out = torch.empty((height, width, 4), dtype=torch.float32, device=f"cuda:{self.device or 0}")
        assert out.is_cuda and out.dtype == torch.float32 and out.is_contiguous() and out.numel() == width * height * 4
        if stream is None:
            stream = torch.cuda.current_stream(out.device).cuda_stream
        check(lib().gs_render(self._h, _mat16(view), _mat16(proj), int(width), int(height), C.c_void_p(out.data_ptr()),
                              1, C.c_void_p(stream)), "gs_render")
        return out

    def render_bgra8(self, view, proj, width: int, height: int, out=None, stream=None):
        """Render as BGRA8Unorm (the reference's drawable format) into `out`
        (torch uint8 CUDA tensor (H, W, 4), bytes B, G, R, A); returns it."""
        import torch

        if out is None:
            out = torch.empty((height, width, 4), dtype=torch.uint8, device=f"cuda:{self.device or 0}")
        assert out.is_cuda and out.dtype == torch.uint8 and out.is_contiguous() and out.numel() == width * height * 4
        if stream is None:
            stream = torch.cuda.current_stream(out.device).cuda_stream
        check(lib().gs_render_bgra8(self._h, _mat16(view), _mat16(proj), int(width), int(height),
                                    C.c_void_p(out.data_ptr()), 1, C.c_void_p(stream)), "gs_render_bgra8")
        return out

    def render_bgra8_host(self, view, proj, width: int, height: int) -> np.ndarray:
        out = np.empty((height, width, 4), np.uint8)
        check(lib().gs_render_bgra8(self._h, _mat16(view), _mat16(proj), int(width), int(height), out.ctypes.data,
                                    0, None), "gs_render_bgra8")
        return out

    def render_host(self, view, proj, width: int, height: int) -> np.ndarray:
        out = np.empty((height, width, 4), np.float32)
        check(lib().gs_render(self._h, _mat16(view), _mat16(proj), int(width), int(height), out.ctypes.data, 0, None),
              "gs_render")
        return out

    def last_stats(self) -> dict:
        s = GsStats()
        check(lib().gs_last_stats(self._h, C.byref(s)), "gs_last_stats")
        return s.as_dict()

    def kernel_times(self, max_frames: int = 64):
        """stage_timing 2: (ms_preprocess, ms_composite) arrays of the last
        frames (<= 64, oldest first) from the events in the kernels' dispatch packets."""
        pre = np.zeros(max_frames, np.float32)
        comp = np.zeros(max_frames, np.float32)
        cnt = C.c_int32(0)
        check(lib().gs_kernel_times(self._h, int(max_frames), pre.ctypes.data_as(C.POINTER(C.c_float)),
                                    comp.ctypes.data_as(C.POINTER(C.c_float)), C.byref(cnt)), "gs_kernel_times")
        return pre[:cnt.value], comp[:cnt.value]

    def project_host(self, view, proj, width: int, height: int):
        n = self.getPointCount()
        rec = np.zeros(n, RECORD_DTYPE)
        dk = np.zeros(n, np.uint32)
        nt = np.zeros(n, np.uint32)
        check(lib().gs_project_host(self._h, _mat16(view), _mat16(proj), int(width), int(height), rec.ctypes.data,
                                    dk.ctypes.data, nt.ctypes.data), "gs_project_host")
        return rec, dk, nt

    def sorted_pairs(self):
        cnt = C.c_int64(0)
        check(lib().gs_sorted_pairs_host(self._h, None, None, 0, C.byref(cnt)), "gs_sorted_pairs_host")
        k = np.zeros(cnt.value, np.uint32)
        v = np.zeros(cnt.value, np.uint32)
        check(lib().gs_sorted_pairs_host(self._h, k.ctypes.data, v.ctypes.data, cnt.value, C.byref(cnt)),
              "gs_sorted_pairs_host")
        return k, v

    def scene(self) -> Scene:
        """The loaded (post-crop) scene as host SoA arrays (gs_get_scene)."""
        n = self.getPointCount()
        a = {k: np.empty(shape, np.float32) for k, shape in
             (("pos", (n, 3)), ("rot", (n, 4)), ("scale", (n, 3)), ("opacity", (n,)), ("color", (n, 3)),
              ("sh_rest", (n, 45)))}
        check(lib().gs_get_scene(self._h, *(a[k].ctypes.data for k in ("pos", "rot", "scale", "opacity", "color",
                                                                         "sh_rest"))), "gs_get_scene")
        return Scene(**a)

    def subset(self, begin: int, end: int) -> "InstancedSplatRenderer":
        """A renderer over splats [begin, end) of this one's scene (gs_create_subset)."""
        r = InstancedSplatRenderer.__new__(InstancedSplatRenderer)
        r.options = Options(**vars(self.options))
        r._h = C.c_void_p()
        r.device = None
        check(lib().gs_create_subset(self._h, int(begin), int(end), C.byref(r._h)), "gs_create_subset")
        return r

    def close(self):
        if self._h:
            lib().gs_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def radix_sort_pairs(keys, vals, bits: int, stream=None):
    """Stable LSD sort of torch uint32-as-int32 CUDA tensors in place."""
    import torch

    n = keys.numel()
    tk = torch.empty_like(keys)
    tv = torch.empty_like(vals)
    if stream is None:
        stream = torch.cuda.current_stream(keys.device).cuda_stream
    check(lib().gs_radix_sort_pairs(C.c_void_p(keys.data_ptr()), C.c_void_p(vals.data_ptr()),
                                    C.c_void_p(tk.data_ptr()), C.c_void_p(tv.data_ptr()), n, int(bits),
                                    C.c_void_p(stream)), "gs_radix_sort_pairs")
    return keys, vals


SCHEMES = {"rows": 0, "slabs": 1, "bands": 2}  # gs_scheme
TRANSPORTS = {"auto": 0, "rccl": 1, "copy": 2}  # gs_transport


class ShardedGroup:
    """Multi-GPU frames from one process (gs_create_sharded):
    one contiguous splat-index shard per device, frames into devices[0] by
    the bin-row scheme (bit-identical to one GPU) or the depth-slab scheme;
    RCCL when every rank has its own device, peer copies otherwise."""

    def __init__(self, source, num_gpus: int, options: Optional[Options] = None, replicated: bool = False):
        """replicated: every rank holds the whole scene (gs_create_replicated),
        rendering its own bin rows ("bands")."""
        self.options = options or Options()
        self._g = C.c_void_p()
        kind = "replicated" if replicated else "sharded"
        if isinstance(source, InstancedSplatRenderer):
            check(getattr(lib(), f"gs_create_{kind}_from_handle")(source._h, int(num_gpus), C.byref(self._g)),
                  f"gs_create_{kind}_from_handle")
        else:
            opt = self.options.to_c()
            check(getattr(lib(), f"gs_create_{kind}")(str(source).encode(), C.byref(opt), int(num_gpus),
                                                       C.byref(self._g)), f"gs_create_{kind}")
        self.device = None

    def initialize(self, devices=None, transport: str = "auto") -> bool:
        arr = None
        if devices is not None:
            d = np.ascontiguousarray(devices, np.int32)
            assert d.shape == (self.size,)
            arr = d.ctypes.data
            self._devices = d
        check(lib().gs_group_initialize(self._g, arr, TRANSPORTS[transport]), "gs_group_initialize")
        self.device = int(devices[0]) if devices is not None else 0
        return True

    @property
    def size(self) -> int:
        return int(lib().gs_group_size(self._g))

    @property
    def transport(self) -> str:
        t = int(lib().gs_group_transport(self._g))
        return {v: k for k, v in TRANSPORTS.items()}.get(t, "none")

    def getPointCount(self) -> int:
        return int(lib().gs_group_point_count(self._g))

    def set_scheme(self, scheme: str):
        check(lib().gs_group_set_scheme(self._g, SCHEMES[scheme]), "gs_group_set_scheme")

    def set_timeout(self, timeout_ms: int):
        """Bound of every host wait (gs_group_set_timeout): an expired wait or
        an RCCL peer error aborts the communicators and raises (GS_ERR_COMM)."""
        check(lib().gs_group_set_timeout(self._g, int(timeout_ms)), "gs_group_set_timeout")

    def render(self, view, proj, width: int, height: int, out=None, stream=None):
        import torch

        if out is None:
            out = torch.empty((height, width, 4), dtype=torch.float32, device=f"cuda:{self.device or 0}")
        assert out.is_cuda and out.dtype == torch.float32 and out.is_contiguous() and out.numel() == width * height * 4
        if stream is None:
            stream = torch.cuda.current_stream(out.device).cuda_stream
        check(lib().gs_group_render(self._g, _mat16(view), _mat16(proj), int(width), int(height),
                                    C.c_void_p(out.data_ptr()), 1, C.c_void_p(stream)), "gs_group_render")
        return out

    def render_host(self, view, proj, width: int, height: int) -> np.ndarray:
        out = np.empty((height, width, 4), np.float32)
        check(lib().gs_group_render(self._g, _mat16(view), _mat16(proj), int(width), int(height), out.ctypes.data,
                                    0, None), "gs_group_render")
        return out

    def set_frames_in_flight(self, n: int):
        """2: rows frames pipelined (gs_group_render_pipelined), one frame's
        all-to-all under the previous frame's render and gather."""
        check(lib().gs_group_set_frames_in_flight(self._g, int(n)), "gs_group_set_frames_in_flight")

    def render_pipelined(self, view, proj, width: int, height: int, out=None, stream=None, host: bool = False):
        """Projects this view's frame and returns the PREVIOUS call's frame
        (None on the first call): a device tensor on the caller's stream, or
        with host=True a numpy array.  flush() returns the last one."""
        return self._pipelined(view, proj, width, height, out, stream, host)

    def flush(self, width: int = 0, height: int = 0, out=None, stream=None, host: bool = False):
        """The frame still in flight (None when there is none); its size is
        the one it was projected at."""
        return self._pipelined(None, None, width, height, out, stream, host)

    def _pipelined(self, view, proj, width, height, out, stream, host):
        import torch

        produced = C.c_int32(0)
        # (the frame that comes back is the one in flight: its size, not this view's)
        prev = getattr(self, "_inflight", None)
        self._inflight = (width, height) if view is not None else None
        ow, oh = prev if prev is not None else (width, height)
        if host:
            buf = np.empty((oh, ow, 4), np.float32)
            ptr, dev_out, st = buf.ctypes.data, 0, None
        else:
            if out is None:
                out = torch.empty((oh, ow, 4), dtype=torch.float32, device=f"cuda:{self.device or 0}")
            assert out.is_cuda and out.dtype == torch.float32 and out.is_contiguous()
            assert out.numel() >= ow * oh * 4, "out holds the frame in flight (the previous call's size)"
            buf, ptr, dev_out = out, out.data_ptr(), 1
            st = stream if stream is not None else torch.cuda.current_stream(out.device).cuda_stream
        if view is None:
            check(lib().gs_group_flush(self._g, C.c_void_p(ptr), dev_out, C.c_void_p(st), C.byref(produced)),
                  "gs_group_flush")
        else:
            check(lib().gs_group_render_pipelined(self._g, _mat16(view), _mat16(proj), int(width), int(height),
                                                  C.c_void_p(ptr), dev_out, C.c_void_p(st), C.byref(produced)),
                  "gs_group_render_pipelined")
        return buf if produced.value else None

    def last_stats(self, rank: int = 0) -> dict:
        s = GsStats()
        check(lib().gs_group_last_stats(self._g, int(rank), C.byref(s)), "gs_group_last_stats")
        return s.as_dict()

    def close(self):
        if self._g:
            lib().gs_group_destroy(self._g)
            self._g = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
