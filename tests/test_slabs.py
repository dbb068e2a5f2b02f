"""Depth-slab multi-GPU scheme on CPU:
slab bounds (gs_slab_bounds, host code of the product library), the oracle's
slab decomposition against its own full composite, and the gloo protocol
(histogram all-reduce, record all-to-all, transmittance all-gather, RGBA
reduce).  The decomposition reassociates the transmittance product, so the
scheme is approximate: the bar is the north star's 1e-4 per channel on all
but a handful of pixels whose A >= 0.99 / T < 0.01 break flips, each bounded
by the 0.01 left at the break (conftest.check_slab_frame); world 1 is
bit-exact."""
import os
import socket

import numpy as np
import pytest

from oracle import oracle_py as O

from conftest import SLAB_FLIP_BOUND, SLAB_FLIP_SHARE, check_slab_frame

TOL = 1e-4


def _flips_ok(got, ref):
    d = np.abs(got.astype(np.float64) - ref.astype(np.float64)).max(axis=-1)
    bad = int((d > TOL).sum())
    return bad, float(d.max()) if d.size else 0.0, d.size


def test_slab_bounds_properties():
    from gaussian_splat_amd.distributed import SLAB_BIN_KEYS, SLAB_BINS, slab_bounds
    rng = np.random.default_rng(0)
    keys_total = SLAB_BINS * SLAB_BIN_KEYS
    for world in (1, 2, 3, 5, 8, 32):
        for trial in range(5):
            h = np.zeros(SLAB_BINS, np.uint64)
            bins = rng.integers(0x300, 0x7C0, size=200)
            np.add.at(h, bins, rng.integers(1, 1000, size=200).astype(np.uint64))
            b = slab_bounds(h, world)
            assert b[0] == 0 and b[-1] == keys_total and np.all(np.diff(b.astype(np.int64)) >= 0)
            assert np.all(b % SLAB_BIN_KEYS == 0)
            cum = np.concatenate([[0], np.cumsum(h.astype(np.int64))])
            tot = cum[-1]
            for d in range(world):
                pairs = cum[b[d + 1] // SLAB_BIN_KEYS] - cum[b[d] // SLAB_BIN_KEYS]
                assert pairs <= tot / world + h.max() + 1  # within one histogram bin of equal shares
    assert slab_bounds(np.zeros(SLAB_BINS, np.uint64), 4).tolist() == [0, 0, 0, 0, keys_total]


def _split(rec, dk, nt, bounds):
    vis = nt > 0
    slab = np.searchsorted(np.asarray(bounds[1:-1], np.int64), dk.astype(np.int64), side="right")
    return [(rec[vis & (slab == d)], dk[vis & (slab == d)]) for d in range(len(bounds) - 1)]


@pytest.mark.parametrize("mode", ["tile", "live50"])
def test_oracle_slab_decomposition(mode):
    from gaussian_splat_amd import scene as S
    from gaussian_splat_amd.api import default_camera
    from gaussian_splat_amd.distributed import SLAB_BIN_KEYS, SLAB_BINS, slab_bounds
    w, h = 320, 200
    sc = S.synthetic_scene(40000, seed=5, sh_degree=0, aspect=w / h)
    cam = default_camera(w, h)
    V, P = cam.getViewMatrix(), cam.getProjectionMatrix()
    rec, dk, nt = O.project(sc, V, P, w, h)
    vis = nt > 0
    full = O.composite_records(rec[vis], dk[vis], w, h, mode=mode)
    hist = np.bincount(dk[vis] // SLAB_BIN_KEYS, weights=nt[vis], minlength=SLAB_BINS).astype(np.uint64)
    for world in (1, 2, 3, 4):
        parts = _split(rec, dk, nt, slab_bounds(hist, world))
        ts = np.stack([O.composite_slab(r, k, w, h, 1, mode=mode) for r, k in parts])
        frame = np.zeros((h, w, 4), np.float32)
        for d, (r, k) in enumerate(parts):
            frame += O.composite_slab(r, k, w, h, 2, rank=d, t_all=ts, mode=mode)
        if world == 1:
            np.testing.assert_array_equal(frame.view(np.uint32), full.view(np.uint32))
        check_slab_frame(frame, full)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, w, h, mode, q):
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent))
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    import torch.distributed as dist
    from cpu_shard_backend import OracleSlabBackend
    from gaussian_splat_amd import scene as S
    from gaussian_splat_amd.api import default_camera
    from gaussian_splat_amd.distributed import SlabRenderer, shard_bounds

    os.environ["OMP_NUM_THREADS"] = "2"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        sc = S.synthetic_scene(n, seed=23, sh_degree=0, aspect=w / h)
        cam = default_camera(w, h)
        cam.orbit(-0.2, 0.1)
        V, P = cam.getViewMatrix(), cam.getProjectionMatrix()
        b, e = shard_bounds(n, world, rank)
        be = OracleSlabBackend(sc.subset(slice(b, e)), rank, world, b, mode=mode)
        frame = SlabRenderer(be, rank, world).render(V, P, w, h)
        if rank == 0:
            ref, _ = O.render(sc, V, P, w, h, mode=mode)
            got = frame.numpy()
            q.put((got.shape == ref.shape,) + _flips_ok(got, ref))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,mode", [(2, "tile"), (3, "live50")])
def test_gloo_slab_frame(world, mode):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 30000, 320, 240, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    same_shape, bad, linf, npx = res
    assert same_shape
    assert linf <= SLAB_FLIP_BOUND, f"slab frame error {linf} beyond the flipped-break bound"
    assert bad <= max(2, int(SLAB_FLIP_SHARE * npx)), f"{bad} pixels beyond 1e-4 (max {linf})"
