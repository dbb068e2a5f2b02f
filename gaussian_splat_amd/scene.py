"""Seeded synthetic scenes with 3DGS statistics and a 3DGS .ply writer.

Positions are uniform in volume inside the default camera's frustum at
zFront in [1, 9] and inside the reference's crop cube (|x|,|y|,|z| < 5,
instanced_splat_renderer.mm:382-386), so every generated splat survives the
crop.  log-scale ~ N(ln 0.01, 0.4), q ~ N(0, I4) (w,x,y,z, raw),
opacity-logit ~ N(0, 1.5), f_dc ~ N(0, 1), f_rest ~ N(0, 0.1).
"""
from __future__ import annotations

import math
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
    f_rest: np.ndarray
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


def synthetic_raw(n: int, seed: int = 0, aspect: float = 16 / 9, fov_deg: float = 45.0,
                  eye=(0.0, 2.0, 5.0), target=(0.0, 0.0, 0.0), up=(0.0, -1.0, 0.0), zrange=(1.0, 9.0),
                  crop: float = 5.0) -> RawSplats:
    rng = np.random.default_rng(seed)
    s, u, f = _view_basis(eye, target, up)
    eye = np.asarray(eye, np.float64)
    t = math.tan(math.radians(fov_deg) / 2)
    z0, z1 = zrange
    pos = np.empty((0, 3), np.float64)
    while pos.shape[0] < n:
        m = int((n - pos.shape[0]) * 1.6) + 1024
        z = np.cbrt(rng.random(m) * (z1 ** 3 - z0 ** 3) + z0 ** 3)  # uniform in volume
        x = (rng.random(m) * 2 - 1) * z * t * aspect
        y = (rng.random(m) * 2 - 1) * z * t
        w = eye + np.outer(x, s) + np.outer(y, u) + np.outer(z, f)
        w = w[np.all(np.abs(w) < crop * 0.999, axis=1)]
        pos = np.concatenate([pos, w])
    pos = pos[:n].astype(np.float32)
    return RawSplats(
        pos=pos,
        f_dc=rng.normal(0.0, 1.0, (n, 3)).astype(np.float32),
        f_rest=rng.normal(0.0, 0.1, (n, 45)).astype(np.float32),
        opacity_logit=rng.normal(0.0, 1.5, n).astype(np.float32),
        log_scale=rng.normal(math.log(0.01), 0.4, (n, 3)).astype(np.float32),
        rot=rng.normal(0.0, 1.0, (n, 4)).astype(np.float32),
    )


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
        col = raw.f_dc.copy()
        rest = raw.f_rest.copy()
    return Scene(pos=raw.pos, rot=raw.rot, scale=sc, opacity=op, color=col, sh_rest=rest)


def synthetic_scene(n: int, seed: int = 0, sh_degree: int = 0, **kw) -> Scene:
    return activate(synthetic_raw(n, seed, **kw), sh_degree)


def write_ply(path, raw: RawSplats, ascii: bool = False, extra_header: Optional[list[str]] = None) -> Path:
    """3DGS 62-property layout (x,y,z,nx,ny,nz,f_dc_0..2,f_rest_0..44,opacity,scale_0..2,rot_0..3)."""
    path = Path(path)
    n = raw.n
    cols = np.concatenate([raw.pos, np.zeros((n, 3), np.float32), raw.f_dc, raw.f_rest,
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
