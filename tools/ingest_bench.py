#!/usr/bin/env python3
"""Scene ingest timing: PLY file -> splats resident in HBM.

  python tools/ingest_bench.py --splats 6000000 [--sh 3] [--dir /tmp/x] [--keep]

Writes a binary 3DGS PLY (62 properties, seeded synthetic values, a tenth
outside the crop box), then times in fresh processes, page cache warm:
  reference    the reference's own PLYLoader::load (oracle/_ref, compiled
               unchanged from src/ply_loader.cpp; one thread, 248-B PointData)
  pointdata    gs_create with GS_PLY_DIRECT=0: the PLYLoader drop-in (bulk read,
               threaded conversion) -> PointData -> crop -> host planes
  direct       gs_create: mmap + parallel conversion straight into the HBM
               planes (scene_io.cpp)
and gs_initialize (host planes -> HBM) for the product paths.  Prints JSON.
"""
import argparse
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def write(path, n, seed, chunk=2_000_000):
    import numpy as np

    from gaussian_splat_amd import scene as S
    hdr = ["ply", "format binary_little_endian 1.0", f"element vertex {n}"]
    hdr += [f"property float {p}" for p in S.PLY_PROPS] + ["end_header"]
    with open(path, "wb") as fh:
        fh.write(("\n".join(hdr) + "\n").encode())
        for b in range(0, n, chunk):
            e = min(n, b + chunk)
            raw = S.synthetic_raw(n, seed=seed, rest=True, start=b, stop=e)
            raw.pos[::10] *= 3.0
            m = e - b
            cols = np.concatenate([raw.pos, np.zeros((m, 3), np.float32), raw.f_dc, raw.f_rest,
                                   raw.opacity_logit[:, None], raw.log_scale, raw.rot], axis=1)
            fh.write(cols.astype("<f4").tobytes())
            print(f"[ingest] wrote {e}/{n}", file=sys.stderr, flush=True)


def child(kind, path, sh):
    out = {}
    if kind == "reference":
        import ctypes as C
        lib = C.CDLL(str(ROOT / "oracle" / "_ref" / "libref_ply.so"))
        lib.ref_ply_load.restype = C.c_longlong
        lib.ref_ply_load.argtypes = [C.c_char_p, C.c_void_p, C.c_longlong]
        t = time.perf_counter()
        n = lib.ref_ply_load(str(path).encode(), None, 0)
        out["load_s"] = time.perf_counter() - t
        out["points"] = int(n)
    else:
        import torch

        from gaussian_splat_amd import InstancedSplatRenderer, Options
        torch.zeros(1, device="cuda:0")  # context up before timing
        t = time.perf_counter()
        r = InstancedSplatRenderer(path, Options(sh_degree=sh, crop=True))
        out["load_s"] = time.perf_counter() - t
        t = time.perf_counter()
        r.initialize(0)
        torch.cuda.synchronize()
        out["upload_s"] = time.perf_counter() - t
        out["points"] = r.getPointCount()
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--splats", type=int, default=6_000_000)
    ap.add_argument("--sh", type=int, default=3)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--dir", default=os.environ.get("TMPDIR", "/tmp"))
    ap.add_argument("--keep", action="store_true")
    ap.add_argument("--kinds", default="reference,pointdata,direct")
    ap.add_argument("--child", default="")
    ap.add_argument("--path", default="")
    a = ap.parse_args()
    if a.child:
        return child(a.child, a.path, a.sh)
    path = Path(a.dir) / f"ingest_{a.splats}.ply"
    t = time.perf_counter()
    if not path.exists():
        write(path, a.splats, a.seed)
    res = {"splats": a.splats, "sh_degree": a.sh, "file_bytes": path.stat().st_size,
           "write_s": round(time.perf_counter() - t, 2), "page_cache": "warm (file just written / read)",
           "load_threads": os.environ.get("GS_LOAD_THREADS") or os.environ.get("OMP_NUM_THREADS") or os.cpu_count()}
    try:
        for kind in a.kinds.split(","):
            if kind == "reference" and not (ROOT / "oracle" / "_ref" / "libref_ply.so").exists():
                res[kind] = "oracle/_ref not built"
                continue
            print(f"[ingest] {kind} ...", file=sys.stderr, flush=True)
            env = dict(os.environ)
            if kind == "pointdata":
                env["GS_PLY_DIRECT"] = "0"
            p = subprocess.run([sys.executable, __file__, "--child", kind, "--path", str(path), "--sh", str(a.sh)],
                               capture_output=True, text=True, env=env, timeout=1200)
            if p.returncode != 0:
                res[kind] = f"exit {p.returncode}: {p.stderr[-300:]}"
                continue
            d = json.loads(p.stdout.strip().splitlines()[-1])
            d = {k: round(v, 3) if isinstance(v, float) else v for k, v in d.items()}
            if "load_s" in d:
                d["load_GBps"] = round(res["file_bytes"] / d["load_s"] / 1e9, 2)
            res[kind] = d
    finally:
        if not a.keep:
            path.unlink(missing_ok=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
