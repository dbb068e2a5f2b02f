#!/usr/bin/env python3
"""Generate tests/golden/ (run in the build container, where /root/reference exists).

1. PLY fixtures + the reference's OWN loader output for each (oracle/_ref =
   /root/reference/src/ply_loader.cpp compiled unchanged): tests/golden/ply/.
   These pin row I1 on any machine, including the GPU box.
2. known_answers.json: hand-derived known-answer vectors for C1/K*/S1/A1,
   each computed here in float64 from the cited reference lines, NOT by the
   oracle (the oracle is checked against them).
"""
from __future__ import annotations

import json
import math
import struct
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

from gaussian_splat_amd import scene as S  # noqa: E402
from oracle import oracle_py as O  # noqa: E402

GOLD = ROOT / "tests" / "golden"


def ply_fixtures() -> dict:
    out = GOLD / "ply"
    out.mkdir(parents=True, exist_ok=True)
    cases = {}

    raw = S.synthetic_raw(300, seed=7, aspect=1.0)
    raw.f_dc[::5] = 0.0  # all-zero DC -> colour left 0 (ply_loader.cpp:133)
    raw.pos[::9, 0] += 6.0  # outside the crop cube
    cases["binary_62prop"] = S.write_ply(out / "binary_62prop.ply", raw)

    small = S.synthetic_raw(20, seed=8, aspect=1.0)
    cases["ascii_62prop"] = S.write_ply(out / "ascii_62prop.ply", small, ascii=True)  # 2N quirk

    # only x,y,z,opacity + an unknown property, declared as double (still read as 4 B)
    p = out / "binary_minimal_typed.ply"
    n = 16
    rng = np.random.default_rng(9)
    vals = rng.normal(0, 1, (n, 5)).astype("<f4")
    hdr = ("ply\nformat binary_little_endian 1.0\ncomment typed props are read as 4 bytes\n"
           f"element vertex {n}\nproperty float x\nproperty float y\nproperty double z\n"
           "property float opacity\nproperty uchar confidence\nend_header\n")
    p.write_bytes(hdr.encode() + vals.tobytes())
    cases["binary_minimal_typed"] = p

    # truncated payload: reference keeps stale chunk bytes (ply_loader.cpp:89-95)
    p = out / "binary_truncated.ply"
    full = (out / "binary_62prop.ply").read_bytes()
    p.write_bytes(full[: len(full) - 248 * 37 - 10])
    cases["binary_truncated"] = p

    # f_rest subset and a face element after the vertices
    p = out / "binary_rest_face.ply"
    n = 12
    props = ["x", "y", "z", "f_dc_0", "f_dc_1", "f_dc_2", "f_rest_0", "f_rest_1", "f_rest_44", "f_rest_45",
             "opacity", "scale_0", "scale_1", "scale_2", "rot_0", "rot_1", "rot_2", "rot_3"]
    vals = rng.normal(0, 1, (n, len(props))).astype("<f4")
    hdr = "ply\nformat binary_little_endian 1.0\nelement vertex %d\n" % n
    hdr += "".join(f"property float {q}\n" for q in props)
    hdr += "element face 2\nproperty list uchar int vertex_indices\nend_header\n"
    p.write_bytes(hdr.encode() + vals.tobytes() + b"\x03" + struct.pack("<3i", 0, 1, 2) * 2)
    cases["binary_rest_face"] = p

    # failures: bad magic, zero vertices, CRLF header
    (out / "bad_magic.ply").write_bytes(b"plyx\nformat ascii 1.0\nelement vertex 1\nproperty float x\nend_header\n1\n")
    (out / "zero_vertices.ply").write_bytes(b"ply\nformat ascii 1.0\nelement vertex 0\nproperty float x\nend_header\n")
    (out / "crlf_header.ply").write_bytes(b"ply\r\nformat ascii 1.0\r\nelement vertex 1\r\nproperty float x\r\nend_header\r\n1\r\n")
    for k in ("bad_magic", "zero_vertices", "crlf_header"):
        cases[k] = out / f"{k}.ply"

    meta = {}
    for name, path in cases.items():
        ok, pts = O.ref_ply_load(path)
        np.save(out / f"{name}.ref.npy", pts.astype(np.float32), allow_pickle=False)
        meta[name] = {"ok": bool(ok), "n": int(pts.shape[0])}
    (out / "manifest.json").write_text(json.dumps(meta, indent=1, sort_keys=True))
    return meta


def f32(x):
    return float(np.float32(x))


def known_answers() -> dict:
    ka = {}
    # --- C1: default app camera (main.mm:55-58 -> trackball_camera.mm:136-163) ---
    eye = np.array([0, 2, 5.0])
    f = -eye / np.linalg.norm(eye)
    s = np.cross(f, [0, -1, 0])
    s /= np.linalg.norm(s)
    u = np.cross(s, f)
    V = np.eye(4)
    V[0, :3], V[1, :3], V[2, :3] = s, u, -f
    V[:3, 3] = [-s @ eye, -u @ eye, f @ eye]
    ka["default_view"] = V.tolist()  # rows [-1,0,0,0] [0,-.9284767,.3713907,0] [0,.3713907,.9284767,-5.3851647]
    def persp(fov, aspect, n, fr):
        ys = 1 / math.tan(math.radians(fov) / 2)
        P = np.zeros((4, 4))
        P[0, 0], P[1, 1] = ys / aspect, ys
        P[2, 2], P[2, 3], P[3, 2] = -(fr + n) / (fr - n), -2 * fr * n / (fr - n), -1
        return P
    ka["proj_1080p"] = persp(45, 1920 / 1080, 0.1, 1000).tolist()
    ka["proj_256"] = persp(45, 1.0, 0.1, 1000).tolist()
    ka["fx_1080p"] = persp(45, 1920 / 1080, 0.1, 1000)[0, 0] * 960  # 1303.675
    ka["near_eff"] = 2 * 1000 * 0.1 / (1000 + 0.1)  # z-clip 0 <= z_ndc: zF >= 2fn/(f+n)

    # --- K1-K6: isotropic splat at the origin, default camera, 256x256 ---
    sigma = 0.1
    z = np.linalg.norm(eye)  # zF of the origin
    fx = persp(45, 1.0, 0.1, 1000)[0, 0] * 128
    a = (fx / z) ** 2 * sigma ** 2 + 1e-4
    r = 3 * math.sqrt(a)
    hx = min(r, 1.0117 * r) * 1.0001 + 1
    x0, x1 = math.ceil(128 - hx - 0.5), math.floor(128 + hx - 0.5)
    ka["iso_splat"] = {"pos": [0, 0, 0], "rot": [1, 0, 0, 0], "scale": [sigma] * 3, "width": 256, "height": 256,
                       "zf": z, "a": a, "b": 0.0, "c": a, "r1": r, "r2": r, "cx": 128.0, "cy": 128.0,
                       "ax": 3 / r, "ay": 0.0, "bx": 0.0, "by": 3 / r, "rect": [x0, x0, x1, x1],
                       "ntiles": (x1 // 16 - x0 // 16 + 1) ** 2}

    # --- S1 + A1: composite of fragment lists (depth, r, g, b, alpha) in arrival order ---
    def tile_rule(fr):  # tile.metal:239-266, float32 arithmetic
        order = sorted(range(len(fr)), key=lambda i: (-float(np.float16(fr[i][0])), i))
        A = np.float32(0); C = np.zeros(3, np.float32)
        for i in order:
            d, rr, g, b, al = (np.float32(v) for v in fr[i])
            sa = np.float32(al * (np.float32(1) - A))
            C = (C + np.array([rr, g, b], np.float32) * sa).astype(np.float32)
            A = np.float32(A + sa)
            if A >= np.float32(0.99):
                break
        return [float(C[0]), float(C[1]), float(C[2]), float(A)]

    def live_rule(fr):  # 50layer.metal:197-222
        order = sorted(range(len(fr)), key=lambda i: (-float(np.float16(fr[i][0])), i))
        T = np.float32(1); C = np.zeros(3, np.float32)
        for i in order:
            d, rr, g, b, al = (np.float32(v) for v in fr[i])
            C = (C + np.array([rr, g, b], np.float32) * T).astype(np.float32)
            T = np.float32(T * (np.float32(1) - al))
            if T < np.float32(0.01):
                break
        return [float(C[0]), float(C[1]), float(C[2]), float(1 - T) if fr else 0.0]

    rgb3 = [[2.0, 1, 0, 0, 0.5], [5.0, 0, 1, 0, 0.5], [3.0, 0, 0, 1, 0.5]]
    lists = {
        "survey_rgb": rgb3,  # tile -> (0.125, 0.5, 0.25, 0.875), green (farthest) on top
        "saturate": [[1.0, 1, 1, 1, 0.9], [2.0, 1, 0, 0, 0.9], [3.0, 0, 1, 0, 0.9]],
        "half_tie": [[2.0, 1, 0, 0, 0.4], [2.0004, 0, 1, 0, 0.4], [1.0, 0, 0, 1, 0.4]],  # equal half depth
        "single": [[4.0, 0.2, 0.4, 0.6, 0.3]],
        "empty": [],
    }
    ka["composite"] = {k: {"frags": v, "tile": tile_rule(v) if v else [0, 0, 0, 0],
                           "live50": live_rule(v) if v else [0, 0, 0, 0]} for k, v in lists.items()}
    # cap 32 (tile.metal:7,202): 40 arrivals, only the first 32 are kept
    many = [[1.0 + 0.1 * i, (i % 3 == 0) * 1.0, (i % 3 == 1) * 1.0, (i % 3 == 2) * 1.0, 0.05] for i in range(40)]
    ka["composite"]["cap32"] = {"frags": many, "cap": 32, "tile": tile_rule(many[:32]),
                                "live50": live_rule(many[:32])}
    ka["half_bits"] = {"1.0": 0x3C00, "0.2": 0x3266, "65504.0": 0x7BFF, "65520.0": 0x7C00, "0.0001": 0x068E,
                       "5.3851647": int(np.float16(5.3851647).view(np.uint16)), "1000.0": 0x63D0}
    return ka


if __name__ == "__main__":
    if not O.ref_available():
        sys.exit("oracle/_ref/libref_ply.so missing: run `make -C oracle` where /root/reference exists")
    GOLD.mkdir(parents=True, exist_ok=True)
    print(ply_fixtures())
    (GOLD / "known_answers.json").write_text(json.dumps(known_answers(), indent=1))
    print("wrote", GOLD)
