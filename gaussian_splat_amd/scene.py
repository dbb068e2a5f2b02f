"""Seeded synthetic scenes with 3DGS statistics and a 3DGS .ply writer.

Positions are uniform in volume inside the default camera's frustum at
zFront in [1, 9] and inside the reference's crop cube (|x|,|y|,|z| < 5,
instanced_splat_renderer.mm:382-386), so every generated splat survives the
crop.  log-scale ~ N(ln 0.01, 0.4), q ~ N(0, I4) (w,x,y,z, raw),
opacity-logit ~ N(0, 1.5), f_dc ~ N(0, 1), f_rest ~ N(0, 0.1).
A scene is a sequence of 2^20-splat chunks, chunk k drawn from its own
generator seeded (seed, k): any slice [start, stop) (a rank's shard of a
global scene) is generated alone and equals that slice of the whole.
"""
from __future__ import annotations

import math
import os
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from pathlib import Path
from typing import Optional

import numpy as np

from .api import Scene

SH_C0 = np.float32(0.28209479177387814)

PLY_PROPS = (["x", "y", "z", "nx", "ny", "nz", "f_dc_0", "f_dc_1", "f_dc_2"] + [f"f_rest_{i}" for i in range(45)]
             + ["opacity", "scale_0", "scale_1", "scale_2", "rot_0", "rot_1", "rot_2", "rot_3"])


@dataclass
class RawSplats:
    """Pre-activation 3DGS attributes as stored in a .ply (float32)."""
    pos: np.ndarray
    f_dc: np.ndarray
    f_rest: Optional[np.ndarray]  # None: generated without (SH degree 0 only)
    opacity_logit: np.ndarray
    log_scale: np.ndarray
    rot: np.ndarray

    @property
    def n(self) -> int:
        return int(self.pos.shape[0])


def _view_basis(eye, target, up):
    f = np.asarray(target, np.float64) - np.asarray(eye, np.float64)
    f /= np.linalg.norm(f)
    s = np.cross(f, up)
    s /= np.linalg.norm(s)
    u = np.cross(s, f)
    return s, u, f


CHUNK = 1 << 20  # splats per independently seeded generator chunk


def _chunk(k: int, m: int, seed: int, aspect: float, fov_deg: float, eye, target, up, zrange, crop: float,
           rest: bool, profile: str):
    """Chunk k (m splats) of a scene: its own generator seeded (seed, k), so a
    slice of the scene is the same whoever generates it (a rank its shard)."""
    rng = np.random.default_rng([seed, k])
    s, u, f = _view_basis(eye, target, up)
    e = np.asarray(eye, np.float64)
    t = math.tan(math.radians(fov_deg) / 2)
    z0, z1 = zrange
    pos = np.empty((0, 3), np.float64)
    while pos.shape[0] < m:
        c = int((m - pos.shape[0]) * 1.6) + 1024
        z = np.cbrt(rng.random(c) * (z1 ** 3 - z0 ** 3) + z0 ** 3)  # uniform in volume
        x = (rng.random(c) * 2 - 1) * z * t * aspect
        y = (rng.random(c) * 2 - 1) * z * t
        w = e + np.outer(x, s) + np.outer(y, u) + np.outer(z, f)
        w = w[np.all(np.abs(w) < crop * 0.999, axis=1)]
        pos = np.concatenate([pos, w])
    pos = pos[:m].astype(np.float32)
    f_dc = rng.standard_normal((m, 3), dtype=np.float32)
    op = rng.standard_normal(m, dtype=np.float32) * np.float32(1.5)
    ls = rng.standard_normal((m, 3), dtype=np.float32) * np.float32(0.4) + np.float32(math.log(0.01))
    if profile == "heavy":
        # heavy-tailed scales (real 3DGS captures): 6 % of the splats 3-20x
        # larger, anisotropic, plus a 1 % tail of large background splats
        big = rng.random(m) < 0.06
        ls[big] += rng.standard_normal((int(big.sum()), 3), dtype=np.float32) * np.float32(0.5) + np.float32(1.6)
        huge = rng.random(m) < 0.01
        ls[huge] += np.float32(1.2)
    elif profile != "uniform":
        raise ValueError("profile must be 'uniform' or 'heavy'")
    rot = rng.standard_normal((m, 4), dtype=np.float32)
    fr = rng.standard_normal((m, 45), dtype=np.float32) * np.float32(0.1) if rest else None
    return pos, f_dc, fr, op, ls, rot


def synthetic_raw(n: int, seed: int = 0, aspect: float = 16 / 9, fov_deg: float = 45.0,
                  eye=(0.0, 2.0, 5.0), target=(0.0, 0.0, 0.0), up=(0.0, -1.0, 0.0), zrange=(1.0, 9.0),
                  crop: float = 5.0, rest: bool = True, profile: str = "uniform", start: int = 0,
                  stop: Optional[int] = None) -> RawSplats:
    """Splats [start, stop) of an n-splat seeded scene (SURVEY §8d statistics).
    rest=False leaves f_rest out (SH degree 0 scenes; f_rest is None).
    profile "heavy": log-scale tail of large splats (scale-stress variant)."""
    stop = n if stop is None else stop
    if not 0 <= start <= stop <= n:
        raise ValueError("bad slice")
    def one(k):
        c0, c1 = k * CHUNK, min(n, (k + 1) * CHUNK)
        a, b = max(start, c0) - c0, min(stop, c1) - c0
        return [None if v is None else v[a:b]
                for v in _chunk(k, c1 - c0, seed, aspect, fov_deg, eye, target, up, zrange, crop, rest, profile)]

    ks = range(start // CHUNK, (stop + CHUNK - 1) // CHUNK)
    # chunks are independent (numpy's generators release the GIL while filling)
    workers = min(len(ks), 16, os.cpu_count() or 1)
    if workers > 1:
        with ThreadPoolExecutor(max_workers=workers) as ex:
            parts = list(ex.map(one, ks))
    else:
        parts = [one(k) for k in ks]
    if not parts:
        z = np.zeros((0, 3), np.float32)
        return RawSplats(pos=z, f_dc=z.copy(), f_rest=np.zeros((0, 45), np.float32) if rest else None,
                         opacity_logit=np.zeros(0, np.float32), log_scale=z.copy(), rot=np.zeros((0, 4), np.float32))
    cat = [None if parts[0][j] is None else np.concatenate([p[j] for p in parts]) for j in range(6)]
    return RawSplats(pos=cat[0], f_dc=cat[1], f_rest=cat[2], opacity_logit=cat[3], log_scale=cat[4], rot=cat[5])


def activate(raw: RawSplats, sh_degree: int = 0) -> Scene:
    """Loader activations (ply_loader.cpp:116-119,132-139) in float32.

    sh_degree 0 -> color = clamp(0.5 + C0 f_dc) with the all-zero skip;
    sh_degree > 0 -> color = raw f_dc and sh_rest = f_rest.
    """
    op = (np.float32(1) / (np.float32(1) + np.exp(-raw.opacity_logit))).astype(np.float32)
    sc = np.exp(raw.log_scale).astype(np.float32)
    if sh_degree == 0:
        col = np.clip(np.float32(0.5) + SH_C0 * raw.f_dc, 0, 1).astype(np.float32)
        zero = np.all(raw.f_dc == 0, axis=1)
        col[zero] = 0
        rest = None
    else:
        if raw.f_rest is None:
            raise ValueError("sh_degree > 0 needs f_rest (synthetic_raw(rest=True))")
        col = raw.f_dc.copy()
        rest = raw.f_rest.copy()
    return Scene(pos=raw.pos, rot=raw.rot, scale=sc, opacity=op, color=col, sh_rest=rest)


def synthetic_scene(n: int, seed: int = 0, sh_degree: int = 0, **kw) -> Scene:
    kw.setdefault("rest", sh_degree > 0)
    return activate(synthetic_raw(n, seed, **kw), sh_degree)


def write_ply(path, raw: RawSplats, ascii: bool = False, extra_header: Optional[list[str]] = None) -> Path:
    """3DGS 62-property layout (x,y,z,nx,ny,nz,f_dc_0..2,f_rest_0..44,opacity,scale_0..2,rot_0..3)."""
    path = Path(path)
    n = raw.n
    fr = raw.f_rest if raw.f_rest is not None else np.zeros((n, 45), np.float32)
    cols = np.concatenate([raw.pos, np.zeros((n, 3), np.float32), raw.f_dc, fr,
                           raw.opacity_logit[:, None], raw.log_scale, raw.rot], axis=1).astype(np.float32)
    hdr = ["ply", f"format {'ascii' if ascii else 'binary_little_endian'} 1.0", f"element vertex {n}"]
    hdr += [f"property float {p}" for p in PLY_PROPS]
    hdr += list(extra_header or [])
    hdr += ["end_header"]
    with open(path, "wb") as fh:
        fh.write(("\n".join(hdr) + "\n").encode())
        if ascii:
            for row in cols:
                fh.write((" ".join(repr(float(v)) for v in row) + "\n").encode())
        else:
            fh.write(cols.astype("<f4").tobytes())
    return path
