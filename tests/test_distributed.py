"""Multi-rank protocol on CPU with gloo: splat-index shards, bin-row
ownership, all_to_all record exchange, band gather + assembly.  The
assembled frame must equal the single-process oracle frame bit for bit."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, w, h, sh, mode, cap, q):
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent))
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    import torch.distributed as dist
    from cpu_shard_backend import OracleShardBackend
    from gaussian_splat_amd import scene as S
    from gaussian_splat_amd.api import default_camera
    from gaussian_splat_amd.distributed import ShardedRenderer, shard_bounds

    os.environ["OMP_NUM_THREADS"] = "2"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        sc = S.synthetic_scene(n, seed=17, sh_degree=sh, aspect=w / h)
        if cap:
            sc.scale *= 3.0
        cam = default_camera(w, h)
        cam.orbit(0.3, 0.05)
        V, P = cam.getViewMatrix(), cam.getProjectionMatrix()
        b, e = shard_bounds(n, world, rank)
        be = OracleShardBackend(sc.subset(slice(b, e)), rank, world, b, sh_degree=sh, mode=mode, cap=cap)
        frame = ShardedRenderer(be, rank, world).render(V, P, w, h)
        if rank == 0:
            from oracle import oracle_py as O
            ref, _ = O.render(sc, V, P, w, h, sh_degree=sh, mode=mode, cap=cap)
            got = frame.numpy()
            q.put((got.shape == ref.shape and bool(np.array_equal(got.view(np.uint32), ref.view(np.uint32))),
                   float(np.abs(got - ref).max()) if got.shape == ref.shape else -1.0))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,sh,mode,cap", [(2, 0, "tile", 0), (3, 3, "tile", 0), (2, 0, "live50", 0),
                                               (3, 0, "tile", 32)])
def test_gloo_sharded_frame_bitexact(world, sh, mode, cap):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 30000, 320, 400, sh, mode, cap, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    same, linf = res
    assert same, f"sharded frame differs from single-process oracle (L-inf {linf})"


def _pipe_worker(rank, world, port, n, w, h, q):
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent))
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    import torch.distributed as dist
    from cpu_shard_backend import OracleShardBackend
    from gaussian_splat_amd import scene as S
    from gaussian_splat_amd.api import default_camera
    from gaussian_splat_amd.distributed import ShardedRenderer, shard_bounds

    os.environ["OMP_NUM_THREADS"] = "2"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        sc = S.synthetic_scene(n, seed=23, sh_degree=0, aspect=w / h)
        cam = default_camera(w, h)
        views = []
        for _ in range(3):
            views.append((cam.getViewMatrix(), cam.getProjectionMatrix()))
            cam.orbit(0.4, 0.05)
        b, e = shard_bounds(n, world, rank)
        xg = dist.new_group(backend="gloo")  # the exchange's own communicator
        sr = ShardedRenderer(OracleShardBackend(sc.subset(slice(b, e)), rank, world, b), rank, world,
                             pipeline=True, exchange_group=xg)
        outs = [sr.render(V, P, w, h) for V, P in views] + [sr.flush(), sr.flush()]
        if rank == 0:
            from oracle import oracle_py as O
            ok = outs[0] is None and outs[4] is None  # one frame of latency; nothing left after the flush
            worst = 0.0
            for k, (V, P) in enumerate(views):
                ref, _ = O.render(sc, V, P, w, h)
                got = outs[k + 1].numpy()
                ok = ok and got.shape == ref.shape and bool(np.array_equal(got.view(np.uint32), ref.view(np.uint32)))
                worst = max(worst, float(np.abs(got - ref).max()) if got.shape == ref.shape else -1.0)
            q.put((ok, worst))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_pipelined_rows_bitexact(world):
    """Pipelined row frames (two in flight, the exchange on its own group):
    call k returns frame k-1, flush() the last; each equals the oracle frame
    of its own view bit for bit."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipe_worker, args=(r, world, port, 20000, 256, 192, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    same, linf = res
    assert same, f"pipelined sharded frames differ from the oracle (L-inf {linf})"


def _band_worker(rank, world, port, n, w, h, sh, mode, q):
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent))
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    import torch.distributed as dist
    from cpu_shard_backend import OracleBandBackend
    from gaussian_splat_amd import scene as S
    from gaussian_splat_amd.api import default_camera
    from gaussian_splat_amd.distributed import BandRenderer

    os.environ["OMP_NUM_THREADS"] = "2"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        sc = S.synthetic_scene(n, seed=19, sh_degree=sh, aspect=w / h)
        cam = default_camera(w, h)
        cam.orbit(-0.2, 0.1)
        V, P = cam.getViewMatrix(), cam.getProjectionMatrix()
        frame = BandRenderer(OracleBandBackend(sc, rank, world, sh_degree=sh, mode=mode), rank, world).render(V, P, w, h)
        if rank == 0:
            from oracle import oracle_py as O
            ref, _ = O.render(sc, V, P, w, h, sh_degree=sh, mode=mode)
            got = frame.numpy()
            q.put((got.shape == ref.shape and bool(np.array_equal(got.view(np.uint32), ref.view(np.uint32))),
                   float(np.abs(got - ref).max()) if got.shape == ref.shape else -1.0))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,sh,mode", [(2, 0, "tile"), (3, 3, "live50")])
def test_gloo_band_frame_bitexact(world, sh, mode):
    """Replicated-scene bands (SURVEY §8(e) fallback): every rank renders its
    owned rows of the whole scene; the gathered frame is the oracle frame."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_band_worker, args=(r, world, port, 20000, 320, 400, sh, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    same, linf = res
    assert same, f"band frame differs from single-process oracle (L-inf {linf})"


def test_assemble_layout():
    import numpy as np
    import torch
    from gaussian_splat_amd.distributed import assemble, band_rows, row_owner
    w, h, world = 40, 140, 3  # 5 bin rows of 32 px (the last partial), owners 0,1,1,2,2
    owner = row_owner(h, world)
    assert owner.tolist() == [0, 1, 1, 2, 2]
    frame = torch.arange(h * w * 4, dtype=torch.float32).view(h, w, 4)
    bands = []
    for r in range(world):
        b = torch.zeros(band_rows(h, world), w, 4)
        for k, ty in enumerate(np.nonzero(owner == r)[0]):
            rows = frame[ty * 32: min(h, ty * 32 + 32)]
            b[k * 32: k * 32 + rows.shape[0]] = rows
        bands.append(b)
    torch.testing.assert_close(assemble(bands, w, h, world), frame, rtol=0, atol=0)
    custom = np.array([2, 1, 0, 1, 2], np.uint8)  # any table works
    bands = []
    for r in range(world):
        b = torch.zeros(band_rows(h, world, custom), w, 4)
        for k, ty in enumerate(np.nonzero(custom == r)[0]):
            rows = frame[ty * 32: min(h, ty * 32 + 32)]
            b[k * 32: k * 32 + rows.shape[0]] = rows
        bands.append(b)
    torch.testing.assert_close(assemble(bands, w, h, world, custom), frame, rtol=0, atol=0)


def _p2p_gather_worker(rank, world, port, w, h, q):
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    import numpy as np
    import torch
    import torch.distributed as dist
    from gaussian_splat_amd.distributed import band_rows, gather_frame, row_owner

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        frame = torch.arange(h * w * 4, dtype=torch.float32).view(h, w, 4)
        band = torch.full((band_rows(h, world), w, 4), -1.0)  # (padding: never sent)
        for k, ty in enumerate(np.nonzero(row_owner(h, world) == rank)[0]):
            rows = frame[ty * 32: min(h, ty * 32 + 32)]
            band[k * 32: k * 32 + rows.shape[0]] = rows
        got = gather_frame(band, w, h, world, rank, p2p=True)
        if rank == 0:
            q.put(bool(torch.equal(got, frame)))
        else:
            assert got is None
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,w,h", [(3, 40, 140), (3, 24, 40), (2, 16, 96)])
def test_gloo_p2p_band_gather(world, w, h):
    """The RCCL band gather's point-to-point path (each rank's valid rows sent
    straight into rank 0's frame), run with CPU tensors over gloo: ragged last
    bin row, and a rank that owns no row (40 px = 2 bin rows over 3 ranks)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_p2p_gather_worker, args=(r, world, port, w, h, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ok


# ---- failure detection: bounded rendezvous and collectives ----

def _lonely_rank(port, q):
    """Rank 0 of a world of 2 whose peer never starts."""
    import sys
    import time
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    from gaussian_splat_amd.distributed import init_ranks
    t0 = time.time()
    try:
        init_ranks("gloo", 3.0, init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=2)
        q.put(("joined", time.time() - t0))
    except Exception as e:  # the rendezvous must give up
        q.put((type(e).__name__, time.time() - t0))


def test_gloo_peer_never_joins_fails_within_timeout():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_lonely_rank, args=(_free_port(), q))
    p.start()
    try:
        what, dt = q.get(timeout=90)
    finally:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert what != "joined" and dt < 30, (what, dt)


def _stuck_exchange_rank(rank, port, q):
    """Both ranks join; rank 1 then stops answering, rank 0 enters the
    row scheme's record exchange, which must fail within the timeout."""
    import sys
    import time
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    import torch
    import torch.distributed as dist
    from gaussian_splat_amd.distributed import exchange, init_ranks
    init_ranks("gloo", 3.0, init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    if rank == 1:
        time.sleep(8)  # a stuck peer: never enters the all_to_all
        q.put(("peer", 0.0))
        return
    t0 = time.time()
    try:
        exchange(torch.zeros(96, dtype=torch.uint8), [1, 1], 48, 2)
        q.put(("completed", time.time() - t0))
    except Exception as e:
        q.put((type(e).__name__, time.time() - t0))
    dist.destroy_process_group()


def test_gloo_stuck_peer_exchange_fails_within_timeout():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stuck_exchange_rank, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=120) for _ in range(2)]
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    r0 = next(r for r in res if r[0] != "peer")
    assert r0[0] != "completed" and r0[1] < 15, r0
