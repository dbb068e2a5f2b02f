#!/usr/bin/env python3
"""Generate tests/golden/ (run in the build container, where /root/reference exists).

1. PLY fixtures + the reference's OWN loader output for each (oracle/_ref =
   /root/reference/src/ply_loader.cpp compiled unchanged): tests/golden/ply/.
   These pin row I1 on any machine, including the GPU box.
2. known_answers.json: hand-derived known-answer vectors for C1/K*/S1/A1,
   each computed here in float64 from the cited reference lines, NOT by the
   oracle (the oracle is checked against them); `k_pins`: K1-K5 records of
   rotated anisotropic off-axis splats, the eigen branches, the near/far clip
   and N2 colours, from a float64 restatement of tile.metal:40-157 and the
   published 3DGS SH basis (`--known-only` regenerates just this file).
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
    def tile_rule(fr):  # tile.metal:239-266, float32 arithmetic, T = 1 - A
        order = sorted(range(len(fr)), key=lambda i: (-float(np.float16(fr[i][0])), i))
        T = np.float32(1); C = np.zeros(3, np.float32)
        for i in order:
            d, rr, g, b, al = (np.float32(v) for v in fr[i])
            sa = np.float32(al * T)
            C = (C + np.array([rr, g, b], np.float32) * sa).astype(np.float32)
            T = np.float32(T - sa)
            if T <= np.float32(0.01):  # A >= 0.99
                break
        return [float(C[0]), float(C[1]), float(C[2]), float(np.float32(1) - T)]

    def tile_rule_aform(fr, dt):
        # the reference's own form, tile.metal:252-263: sa = alpha (1 - A),
        # C += c sa, A += sa, break at A >= 0.99 (there in half; here in
        # float64 and float32).  Returns (rgba, records composited, the A
        # before each break test).
        order = sorted(range(len(fr)), key=lambda i: (-float(np.float16(fr[i][0])), i))
        A = dt(0); C = np.zeros(3, dt); n = 0; hist = []
        for i in order:
            d, rr, g, b, al = (dt(v) for v in fr[i])
            sa = dt(al * (dt(1) - A))
            C = (C + np.array([rr, g, b], dt) * sa).astype(dt)
            A = dt(A + sa)
            n += 1
            hist.append(float(A))
            if A >= dt(0.99):
                break
        return [float(C[0]), float(C[1]), float(C[2]), float(A)], n, hist

    def tile_count(fr):  # records the T-form contract composites
        order = sorted(range(len(fr)), key=lambda i: (-float(np.float16(fr[i][0])), i))
        T = np.float32(1); n = 0
        for i in order:
            T = np.float32(T - np.float32(np.float32(fr[i][4]) * T))
            n += 1
            if T <= np.float32(0.01):
                break
        return n

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
        "saturate": [[1.0, 1, 1, 1, 0.95], [2.0, 1, 0, 0, 0.95], [3.0, 0, 1, 0, 0.9]],
        # A lands on 0.99 in exact arithmetic: the f32 rounding of the rule decides
        "saturate_edge": [[1.0, 1, 1, 1, 0.9], [2.0, 1, 0, 0, 0.9], [3.0, 0, 1, 0, 0.9]],
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
    # The tile rule's answers in the reference's A-form,
    # beside the T-form contract's.  A case whose break
    # index differs between the forms is a straddle: A lands within 1e-5 of
    # 0.99 there, and the f32 rounding of either form decides.
    for k, c in ka["composite"].items():
        fr = c["frags"][:c["cap"]] if c.get("cap") else c["frags"]
        a64, n64, h64 = tile_rule_aform(fr, np.float64) if fr else ([0, 0, 0, 0], 0, [])
        a32, n32, _ = tile_rule_aform(fr, np.float32) if fr else ([0, 0, 0, 0], 0, [])
        nt = tile_count(fr) if fr else 0
        c["tile_aform64"], c["tile_aform32"] = a64, a32
        c["n_tform"], c["n_aform64"], c["n_aform32"] = nt, n64, n32
        c["straddle"] = bool(nt != n64 or nt != n32)
        if c["straddle"]:  # the A (float64) at the first break test whose outcome differs
            j = min(nt, n64, n32) - 1
            c["straddle_A"] = h64[j]
    ka["half_bits"] = {"1.0": 0x3C00, "0.2": 0x3266, "65504.0": 0x7BFF, "65520.0": 0x7C00, "0.0001": 0x068E,
                       "5.3851647": int(np.float16(5.3851647).view(np.uint16)), "1000.0": 0x63D0}
    return ka


# ---- K1-K5 and N2 pins: a float64 restatement written from the shader lines ----
# Independent of oracle/gs_oracle.c and of DESIGN.md's fp32 contract: matrix
# algebra in float64 straight from gaussian_splat_tile.metal:40-157 (Metal
# matrices are column-major, float3x3(c0, c1, c2) takes COLUMNS, m[col][row]),
# and the published 3DGS real-SH basis (Kerbl et al. 2023, utils/sh_utils.py).
SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
SH_C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
         1.445305721320277, -0.5900435899266435]


def ref64_vertex(pos, rot, scale, V, P, W, H, jz_sign=-1.0):
    """vertex_main (tile.metal:85-157) + the quad's closed form, float64.
    V, P: 4x4 math-convention matrices (M[row, col]).  jz_sign: the sign of
    the Jacobian's z column (-1 = the shader's :122-123; +1 only to show that
    the pins depend on it)."""
    V = np.asarray(V, np.float64)
    P = np.asarray(P, np.float64)
    p4 = np.append(np.asarray(pos, np.float64), 1.0)
    vp = V @ p4                                       # :94  viewMatrix * float4(position, 1)
    zf = -vp[2]                                       # :96-97
    out = {"zf": zf, "visible": False}
    if zf < 1e-4:                                     # :99-105
        out["cull"] = "zfront"
        return out
    q = np.asarray(rot, np.float64)
    w, x, y, z = q / np.linalg.norm(q)                # :41-42 normalize, w = q[0]
    R = np.column_stack([[1 - 2 * (y * y + z * z), 2 * (x * y + w * z), 2 * (x * z - w * y)],
                         [2 * (x * y - w * z), 1 - 2 * (x * x + z * z), 2 * (y * z + w * x)],
                         [2 * (x * z + w * y), 2 * (y * z - w * x), 1 - 2 * (x * x + y * y)]])  # :44-48
    M = R @ np.diag(np.asarray(scale, np.float64))    # :52-58 R * S
    Sigma = M @ M.T                                   # :59
    Wr = V[:3, :3]                                    # :109-113 float3x3(viewMatrix[0..2].xyz)
    Sv = (Wr @ Sigma) @ Wr.T                          # :115
    fx = P[0, 0] * (W * 0.5)                          # :117 projectionMatrix[0][0]
    fy = P[1, 1] * (H * 0.5)                          # :118
    J0 = np.array([fx / zf, 0.0, jz_sign * fx * vp[0] / zf ** 2])  # :120-122
    J1 = np.array([0.0, fy / zf, jz_sign * fy * vp[1] / zf ** 2])  # :123
    a = J0 @ Sv @ J0 + 1e-4                           # :125, :129-130
    b = J0 @ Sv @ J1                                  # :126
    c = J1 @ Sv @ J1 + 1e-4                           # :127, :131
    tr, det = a + c, a * c - b * b                    # eigenSym2x2 :62-83
    s = math.sqrt(max(0.0, 0.25 * tr * tr - det))
    l1, l2 = 0.5 * tr + s, 0.5 * tr - s
    if abs(b) > 1e-8:
        e1 = np.array([l1 - c, b]) / math.hypot(l1 - c, b)
    else:
        e1 = np.array([1.0, 0.0]) if a >= c else np.array([0.0, 1.0])
    e2 = np.array([-e1[1], e1[0]])
    r1, r2 = 3 * math.sqrt(max(l1, 0.0)), 3 * math.sqrt(max(l2, 0.0))  # :133-140
    clip = (P @ V) @ p4                               # :145 viewProjectionMatrix (= P V, .mm:453)
    ndc = clip[:3] / clip[3]                          # :146-147, z = clip.z * invW (:152)
    out.update(a=a, b=b, c=c, r1=r1, r2=r2, e1=e1.tolist(), z_ndc=ndc[2])
    # Metal clips to 0 <= z_ndc <= 1; the fragment stage drops depth < 0.001 (:187)
    if not (0.0 <= ndc[2] <= 1.0):
        out["cull"] = "zclip"
        return out
    if zf < 0.001 or not (r1 > 0 and r2 > 0):
        out["cull"] = "depth/area"
        return out
    # window position of the centre (viewport y down) and the quad's uv = 3 q
    # as a linear function of the pixel offset d = (x - cx, cy - y):
    # uv = (3 d.e1 / r1, 3 d.e2 / r2)  (offsetPx = q.x r1 e1 + q.y r2 e2, :143)
    cx, cy = (ndc[0] + 1) * W / 2, (1 - ndc[1]) * H / 2
    A, B = e1 * 3 / r1, e2 * 3 / r2
    out.update(visible=True, cx=cx, cy=cy, ax=A[0], ay=A[1], bx=B[0], by=B[1])
    return out


def ref64_sh(pos, campos, f_dc, f_rest, deg):
    """eval_sh of the published 3DGS basis, dir = normalize(pos - campos),
    f_rest channel-major (ply f_rest_{ch*15+k}); +0.5 and the loader's [0,1]
    clamp (ply_loader.cpp:11-20; the reference has no SH > 0)."""
    d = np.asarray(pos, np.float64) - np.asarray(campos, np.float64)
    x, y, z = d / np.linalg.norm(d)
    fr = np.asarray(f_rest, np.float64).reshape(3, 15)
    out = []
    for ch in range(3):
        sh = np.concatenate([[f_dc[ch]], fr[ch]])
        r = SH_C0 * sh[0]
        if deg > 0:
            r = r - SH_C1 * y * sh[1] + SH_C1 * z * sh[2] - SH_C1 * x * sh[3]
        if deg > 1:
            xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
            r = (r + SH_C2[0] * xy * sh[4] + SH_C2[1] * yz * sh[5] + SH_C2[2] * (2 * zz - xx - yy) * sh[6]
                 + SH_C2[3] * xz * sh[7] + SH_C2[4] * (xx - yy) * sh[8])
        if deg > 2:
            r = (r + SH_C3[0] * y * (3 * xx - yy) * sh[9] + SH_C3[1] * xy * z * sh[10]
                 + SH_C3[2] * y * (4 * zz - xx - yy) * sh[11] + SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[12]
                 + SH_C3[4] * x * (4 * zz - xx - yy) * sh[13] + SH_C3[5] * z * (xx - yy) * sh[14]
                 + SH_C3[6] * x * (xx - 3 * yy) * sh[15])
        out.append(min(max(r + 0.5, 0.0), 1.0))
    return out


def _f32(a):
    return np.asarray(a, np.float32).astype(np.float64)


def k_pins() -> dict:
    """Splats whose K1-K5 outputs the oracle must reproduce (within fp32
    rounding of these float64 values), by camera."""
    def look_at(eye, tgt, up):
        e, t = np.asarray(eye, np.float64), np.asarray(tgt, np.float64)
        f = (t - e) / np.linalg.norm(t - e)
        s = np.cross(f, up)
        s /= np.linalg.norm(s)
        u = np.cross(s, f)
        V = np.eye(4)
        V[0, :3], V[1, :3], V[2, :3] = s, u, -f
        V[:3, 3] = [-s @ e, -u @ e, f @ e]
        return V

    def persp(fov, aspect, n, fr):
        ys = 1 / math.tan(math.radians(fov) / 2)
        P = np.zeros((4, 4))
        P[0, 0], P[1, 1] = ys / aspect, ys
        P[2, 2], P[2, 3], P[3, 2] = -(fr + n) / (fr - n), -2 * fr * n / (fr - n), -1
        return P

    W, H = 1920, 1080
    cams = {"default": (_f32(look_at([0, 2, 5], [0, 0, 0], [0, -1, 0])), _f32(persp(45, W / H, 0.1, 1000))),
            "axis": (_f32(np.eye(4)), _f32(persp(45, W / H, 0.1, 1000)))}  # eye at 0 looking down -z
    cases = [
        # rotated, anisotropic, off-axis (vx, vy != 0: the J z-column sign matters)
        ("rot_aniso_1", "default", (0.8, -0.5, 1.2), (0.9, 0.3, -0.2, 0.25), (0.05, 0.01, 0.002)),
        ("rot_aniso_2", "default", (-1.5, 0.7, -0.3), (0.2, -0.7, 0.5, 0.4), (0.02, 0.08, 0.01)),
        ("rot_aniso_3", "default", (0.3, 1.1, 2.0), (-0.5, 0.5, 0.5, 0.5), (0.004, 0.03, 0.06)),
        ("rot_aniso_4", "default", (-0.9, -1.2, 0.5), (0.1, 0.2, 0.9, -0.3), (0.1, 0.02, 0.05)),
        ("rot_aniso_5", "default", (1.7, 0.2, -1.0), (0.6, -0.1, -0.6, 0.5), (0.015, 0.015, 0.2)),
        ("rot_aniso_6", "default", (0.05, 0.4, 3.0), (0.3, 0.3, -0.3, 0.85), (0.03, 0.005, 0.012)),
        ("unnormalised_quat", "default", (-0.4, 0.9, -1.6), (2.0, -1.0, 0.6, 1.4), (0.03, 0.012, 0.04)),
        ("edge_straddle", "default", (2.95, -0.2, 0.4), (0.7, 0.1, 0.7, -0.1), (0.4, 0.1, 0.2)),
        # b == 0 exactly (vx = 0, axis-aligned): eigen fallback e1 = (0, 1) if a < c, (1, 0) if a >= c (:77-81)
        ("b0_a_lt_c", "axis", (0.0, 0.7, -5.0), (1.0, 0.0, 0.0, 0.0), (0.01, 0.03, 0.02)),
        ("b0_a_ge_c", "axis", (0.0, 0.7, -5.0), (1.0, 0.0, 0.0, 0.0), (0.03, 0.01, 0.02)),
        # 0 < |b| <= 1e-8 (vx = -6e-9): still the fallback branch
        ("b_tiny_a_lt_c", "axis", (-6e-9, 0.7, -5.0), (1.0, 0.0, 0.0, 0.0), (0.01, 0.03, 0.02)),
        # near plane: Metal's z-clip keeps z_ndc >= 0, i.e. zF >= 2fn/(f+n) = 0.19998
        ("near_in", "axis", (0.01, 0.02, -0.2005), (0.9, 0.2, 0.3, 0.25), (0.001, 0.002, 0.0015)),
        ("near_out", "axis", (0.01, 0.02, -0.1995), (0.9, 0.2, 0.3, 0.25), (0.001, 0.002, 0.0015)),
        ("behind", "axis", (0.0, 0.0, 0.5), (1.0, 0.0, 0.0, 0.0), (0.01, 0.01, 0.01)),
        ("beyond_far", "axis", (0.0, 0.0, -1001.0), (1.0, 0.0, 0.0, 0.0), (1.0, 1.0, 1.0)),
    ]
    out = {"width": W, "height": H, "cameras": {k: {"view": v.tolist(), "proj": p.tolist()} for k, (v, p) in cams.items()},
           "splats": []}
    for name, cam, pos, rot, scale in cases:
        V, P = cams[cam]
        pos, rot, scale = _f32(pos), _f32(rot), _f32(scale)
        r = ref64_vertex(pos, rot, scale, V, P, W, H)
        if name.startswith("rot_aniso"):  # the pin must see the shader's J z-column sign
            alt = ref64_vertex(pos, rot, scale, V, P, W, H, jz_sign=+1.0)
            assert abs(alt["b"] - r["b"]) > 1e-3 * max(abs(r["a"]), abs(r["c"])), name
        out["splats"].append({"name": name, "camera": cam, "pos": pos.tolist(), "rot": rot.tolist(),
                              "scale": scale.tolist(), "expect": r})
    # N2: SH degree 1-3 colours from the published basis
    V, P = cams["default"]
    campos = -(V[:3, :3].T @ V[:3, 3])
    rng = np.random.default_rng(2024)
    sh = []
    for deg in (1, 2, 3):
        for k in range(4):
            pos = _f32(rng.uniform(-1.5, 1.5, 3))
            f_dc = _f32(rng.normal(0, 0.5, 3) if k < 3 else [4.0, -4.0, 0.1])  # k = 3: clamps at 1 and 0
            f_rest = _f32(rng.normal(0, 0.3, 45))
            sh.append({"deg": deg, "pos": pos.tolist(), "f_dc": f_dc.tolist(), "f_rest": f_rest.tolist(),
                       "rgb": ref64_sh(pos, campos, f_dc, f_rest, deg)})
    out["sh"] = sh
    return out


# ---- K6 + F1 (+ S1/A1) per pixel ----
# The float64 raster restatement itself lives in tests/pixel_pins.py (the
# GPU tests evaluate it at the device's own records too); these functions
# build the committed fixtures from it.
sys.path.insert(0, str(ROOT / "tests"))
from pixel_pins import STRADDLE, ref64_quad_alpha  # noqa: E402


def _vertex_alpha(v: dict, opacity: float, W: int, H: int):
    if not v.get("visible"):
        return 0, 0, np.zeros((0, 0)), np.zeros((0, 0), bool)
    return ref64_quad_alpha(v["cx"], v["cy"], v["e1"], v["r1"], v["r2"], v["zf"], opacity, W, H)


def _half(x) -> float:
    return float(np.float16(np.float32(x)))


def ref64_frame(splats: list, W: int, H: int):
    """Tile-rule frame in float64 (tile.metal:239-266): per pixel the covering
    fragments sorted by descending half depth, ties in arrival (index) order,
    then sa = a (1 - A), C += rgb sa, A += sa, break at A >= 0.99.  splats:
    (vertex dict, opacity, rgb).  Returns (rgba[H, W, 4] float64, straddle
    mask[H, W]): a pixel is flagged if any fragment straddles K6/F1 or if A
    lands within STRADDLE of the 0.99 break at some step."""
    frags = [[[] for _ in range(W)] for _ in range(H)]
    strad = np.zeros((H, W), bool)
    for i, (v, op, rgb) in enumerate(splats):
        x0, y0, al, st = _vertex_alpha(v, op, W, H)
        if al.size == 0:
            continue
        strad[y0:y0 + al.shape[0], x0:x0 + al.shape[1]] |= st
        for yy, xx in zip(*np.nonzero(al)):
            frags[y0 + yy][x0 + xx].append((-_half(v["zf"]), i, al[yy, xx], rgb))
    out = np.zeros((H, W, 4))
    for y in range(H):
        for x in range(W):
            A, C = 0.0, np.zeros(3)
            for _, _, a, rgb in sorted(frags[y][x], key=lambda f: (f[0], f[1])):
                sa = a * (1.0 - A)
                C = C + np.asarray(rgb) * sa
                A += sa
                if abs(A - 0.99) < STRADDLE:
                    strad[y, x] = True
                if A >= 0.99:
                    break
            out[y, x, :3], out[y, x, 3] = C, A
    return out, strad


def _look_at64(eye, tgt, up):
    e, t = np.asarray(eye, np.float64), np.asarray(tgt, np.float64)
    f = (t - e) / np.linalg.norm(t - e)
    s = np.cross(f, up)
    s /= np.linalg.norm(s)
    u = np.cross(s, f)
    V = np.eye(4)
    V[0, :3], V[1, :3], V[2, :3] = s, u, -f
    V[:3, 3] = [-s @ e, -u @ e, f @ e]
    return V


def _persp64(fov, aspect, n, fr):
    ys = 1 / math.tan(math.radians(fov) / 2)
    P = np.zeros((4, 4))
    P[0, 0], P[1, 1] = ys / aspect, ys
    P[2, 2], P[2, 3], P[3, 2] = -(fr + n) / (fr - n), -2 * fr * n / (fr - n), -1
    return P


def _half_safe(zf: float) -> bool:
    """zF far enough from a half rounding boundary that fp32 rounding of the
    projection cannot move its S1 key."""
    return _half(zf * (1 - 4e-6)) == _half(zf * (1 + 4e-6))


def pixel_frames() -> dict:
    """Small frames of overlapping rotated splats (SH 0) and their float64
    tile-rule images: name -> dict of arrays for np.savez."""
    specs = [
        # name, W, H, eye, n, scale range (log10), opacity range, seed
        ("rotated_96x64", 96, 64, (0.0, 2.0, 5.0), 40, (-1.6, -0.7), (0.2, 0.98), 11),
        ("needles_128x72", 128, 72, (1.5, 1.0, 4.5), 36, (-2.6, -0.6), (0.3, 0.99), 12),
        ("dense_64x64", 64, 64, (0.0, 0.5, 3.5), 160, (-1.7, -1.0), (0.5, 0.995), 13),
        ("ties_80x80", 80, 80, (0.0, 0.0, 4.0), 24, (-1.4, -0.9), (0.3, 0.9), 14),
    ]
    out = {}
    for name, W, H, eye, n, (lo, hi), (olo, ohi), seed in specs:
        rng = np.random.default_rng(seed)
        V = _f32(_look_at64(eye, [0, 0, 0], [0, -1, 0]))
        P = _f32(_persp64(45, W / H, 0.1, 1000))
        s, u, f = V[0, :3], V[1, :3], -V[2, :3]
        e = np.asarray(eye, np.float64)
        t = math.tan(math.radians(22.5))
        pos, rot, scale, opac, col = [], [], [], [], []
        while len(pos) < n:
            z = rng.uniform(2.5, 6.5)
            p = e + z * f + rng.uniform(-0.8, 0.8) * z * t * (W / H) * s + rng.uniform(-0.8, 0.8) * z * t * u
            if name.startswith("ties") and len(pos) % 6 == 1:
                # same half depth as the previous splat, different fp32 zF:
                # S1's tie goes to the earlier arrival (index)
                p = pos[-1] + rng.uniform(-1e-3, 1e-3) * f + 0.03 * s
            sc = 10 ** rng.uniform(lo, hi, 3)
            if name.startswith("needles"):
                sc[rng.integers(3)] *= 12.0  # long thin splats: the quad's box edge and the cutoff matter
            cand = (_f32(p), _f32(rng.normal(0, 1, 4)), _f32(sc))
            v = ref64_vertex(*cand, V, P, W, H)
            if not v["visible"] or not _half_safe(v["zf"]):
                continue
            if name.startswith("ties") and len(pos) % 6 == 1:
                if _half(v["zf"]) != _half(ref64_vertex(pos[-1], rot[-1], scale[-1], V, P, W, H)["zf"]):
                    continue
            pos.append(cand[0]); rot.append(cand[1]); scale.append(cand[2])
            opac.append(float(np.float32(rng.uniform(olo, ohi))))
            col.append(_f32(rng.uniform(0, 1, 3)))
        splats = [(ref64_vertex(pos[i], rot[i], scale[i], V, P, W, H), opac[i], col[i]) for i in range(n)]
        if name.startswith("ties"):
            assert all(_half(splats[i][0]["zf"]) == _half(splats[i - 1][0]["zf"])
                       and splats[i][0]["zf"] != splats[i - 1][0]["zf"] for i in range(1, n, 6))
        img, strad = ref64_frame(splats, W, H)
        out[name] = {"view": V.astype(np.float32), "proj": P.astype(np.float32), "width": np.int32(W),
                     "height": np.int32(H), "pos": np.array(pos, np.float32), "rot": np.array(rot, np.float32),
                     "scale": np.array(scale, np.float32), "opacity": np.array(opac, np.float32),
                     "color": np.array(col, np.float32), "rgba": img.astype(np.float32),
                     "straddle": strad.astype(np.uint8)}
        print(f"{name}: {W}x{H}, {n} splats, covered {int((img[..., 3] > 0).sum())} px, "
              f"straddling {int(strad.sum())} px")
    return out


def pixel_alpha_pins() -> dict:
    """Per-pixel alpha of every visible k_pin splat over its quad's pixel box
    (1920x1080, opacity 0.7): name -> dict(x0, y0, alpha float32, straddle)."""
    kp = k_pins()
    W, H = kp["width"], kp["height"]
    out = {}
    for sp in kp["splats"]:
        e = sp["expect"]
        if not e["visible"]:
            continue
        x0, y0, al, st = _vertex_alpha(e, float(np.float32(0.7)), W, H)
        out[sp["name"]] = {"x0": np.int32(x0), "y0": np.int32(y0), "alpha": al.astype(np.float32),
                           "straddle": st.astype(np.uint8)}
        print(f"{sp['name']}: box {al.shape[1]}x{al.shape[0]} at ({x0},{y0}), "
              f"{int((al > 0).sum())} covered, {int(st.sum())} straddling")
    return out


def write_pixel_fixtures() -> None:
    d = GOLD / "pixels"
    d.mkdir(parents=True, exist_ok=True)
    for name, arrs in pixel_frames().items():
        np.savez_compressed(d / f"frame_{name}.npz", **arrs)
    pins = pixel_alpha_pins()
    flat = {}
    for name, a in pins.items():
        for k, v in a.items():
            flat[f"{name}__{k}"] = v
    np.savez_compressed(d / "alpha_pins.npz", **flat)
    print("wrote", d)


if __name__ == "__main__":
    if "--pixels" in sys.argv:  # K6 + F1 per-pixel pins (float64), no reference build needed
        write_pixel_fixtures()
        sys.exit(0)
    if "--known-only" in sys.argv:  # the float64 pins need no reference build
        ka = json.loads((GOLD / "known_answers.json").read_text()) if (GOLD / "known_answers.json").exists() else {}
        ka.update(known_answers())
        ka["k_pins"] = k_pins()
        (GOLD / "known_answers.json").write_text(json.dumps(ka, indent=1))
        print("wrote", GOLD / "known_answers.json")
        sys.exit(0)
    if not O.ref_available():
        sys.exit("oracle/_ref/libref_ply.so missing: run `make -C oracle` where /root/reference exists")
    GOLD.mkdir(parents=True, exist_ok=True)
    print(ply_fixtures())
    ka = known_answers()
    ka["k_pins"] = k_pins()
    (GOLD / "known_answers.json").write_text(json.dumps(ka, indent=1))
    print("wrote", GOLD)
