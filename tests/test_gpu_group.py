"""GPU tests of the one-process multi-GPU group (gs_create_sharded, SURVEY
§8(b)/(e)).  On a one-GPU box the ranks are virtual (devices [0, 0, ...],
peer-copy transport): the same gs_shard_* / gs_slab_* steps and buffers as
on 8 GPUs, with hipMemcpyPeerAsync in place of RCCL.  The RCCL transport
runs on real devices when the box has two or more GPUs, and on one GPU
through the test stub of its entry points (test_group_rccl_stub_bitexact).

Bar: the bin-row scheme is bit-identical to the 1-GPU frame; the depth-slab
scheme is bit-identical to the Python virtual-slab path (same passes, same
summation order) and within the slab bound (conftest.check_slab_frame) of
the 1-GPU frame."""
import numpy as np
import pytest

from conftest import check_slab_frame, orbit_views

pytestmark = pytest.mark.gpu


def _scene(n, seed, sh, aspect):
    from gaussian_splat_amd import scene as S
    return S.activate(S.synthetic_raw(n, seed=seed, aspect=aspect, rest=sh > 0), sh)


def _group(r, world, devices=None, transport="copy", scheme="rows"):
    from gaussian_splat_amd import ShardedGroup
    g = ShardedGroup(r, world)
    g.initialize(devices if devices is not None else [0] * world, transport)
    g.set_scheme(scheme)
    return g


@pytest.mark.parametrize("world,mode,sh,W,H", [(2, "tile", 3, 640, 400), (3, "live50", 0, 640, 400),
                                               (4, "tile", 3, 1920, 1080), (1, "tile", 0, 256, 256)])
def test_group_rows_bitexact(built, world, mode, sh, W, H):
    from gaussian_splat_amd import InstancedSplatRenderer, Options
    n = 200000 if W > 1000 else 60000
    sc = _scene(n, 51 + world, sh, W / H)
    r = InstancedSplatRenderer(sc, Options(mode=mode, sh_degree=sh, crop=False))
    r.initialize(0)
    g = _group(r, world)
    assert g.transport == "copy" and g.size == world
    for V, P in orbit_views(W, H, 2):
        ref = r.render_host(V, P, W, H)
        got = g.render_host(V, P, W, H)
        assert int(np.count_nonzero(got.view(np.uint32) != ref.view(np.uint32))) == 0
        dev = g.render(V, P, W, H).cpu().numpy()  # device output, caller's stream
        np.testing.assert_array_equal(dev.view(np.uint32), ref.view(np.uint32))
    st = g.last_stats(0)
    assert st["width"] == W and st["height"] == H


@pytest.mark.parametrize("world,mode,sh", [(2, "tile", 3), (3, "live50", 0)])
def test_group_slabs(built, world, mode, sh):
    from gaussian_splat_amd import InstancedSplatRenderer, Options
    from gaussian_splat_amd import distributed as D
    W, H = 640, 400
    sc = _scene(60000, 61 + world, sh, W / H)
    r = InstancedSplatRenderer(sc, Options(mode=mode, sh_degree=sh, crop=False))
    r.initialize(0)
    g = _group(r, world, scheme="slabs")
    V, P = orbit_views(W, H, 2)[1]
    got = g.render_host(V, P, W, H)
    virt = D.render_virtual_slabs(sc, world, V, P, W, H, sh_degree=sh, mode=mode)
    np.testing.assert_array_equal(got.view(np.uint32), virt.view(np.uint32))
    check_slab_frame(got, r.render_host(V, P, W, H))


def test_group_from_ply_with_crop(built, tmp_path):
    """gs_create_sharded(path): the crop applies to the global scene before
    sharding, so the group's frame is the 1-GPU frame of the same file."""
    from gaussian_splat_amd import InstancedSplatRenderer, Options, ShardedGroup
    from gaussian_splat_amd import scene as S
    raw = S.synthetic_raw(80000, seed=71, aspect=16 / 9, rest=True)
    raw.pos[::5] *= 2.0  # some outside the crop box
    p = S.write_ply(tmp_path / "s.ply", raw)
    W, H = 960, 540
    opt = Options(sh_degree=3, crop=True)
    r = InstancedSplatRenderer(p, opt)
    r.initialize(0)
    g = ShardedGroup(p, 3, opt)
    g.initialize([0, 0, 0], "copy")
    assert g.getPointCount() == r.getPointCount() < 80000
    V, P = orbit_views(W, H, 1)[0]
    np.testing.assert_array_equal(g.render_host(V, P, W, H).view(np.uint32), r.render_host(V, P, W, H).view(np.uint32))


def test_group_rccl_two_gpus(built):
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("RCCL transport needs two GPUs (this box has one)")
    from gaussian_splat_amd import InstancedSplatRenderer, Options
    W, H = 640, 400
    sc = _scene(60000, 81, 0, W / H)
    r = InstancedSplatRenderer(sc, Options(crop=False))
    r.initialize(0)
    from gaussian_splat_amd import ShardedGroup
    for scheme in ("rows", "slabs", "bands"):
        if scheme == "bands":
            g = ShardedGroup(r, 2, replicated=True)
            g.initialize([0, 1], "auto")
        else:
            g = _group(r, 2, devices=[0, 1], transport="auto", scheme=scheme)
        assert g.transport == "rccl"
        V, P = orbit_views(W, H, 1)[0]
        ref = r.render_host(V, P, W, H)
        got = g.render_host(V, P, W, H)
        if scheme in ("rows", "bands"):
            np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))
        else:
            check_slab_frame(got, ref)
        g.close()


_STUB_SCRIPT = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
sys.path.insert(0, sys.argv[1] + "/tests")
from conftest import orbit_views
from gaussian_splat_amd import InstancedSplatRenderer, Options, ShardedGroup
from gaussian_splat_amd import scene as S

def run(world, scheme, mode, sh, W, H, n, seed):
    sc = S.activate(S.synthetic_raw(n, seed=seed, aspect=W / H, rest=sh > 0), sh)
    r = InstancedSplatRenderer(sc, Options(mode=mode, sh_degree=sh, crop=False))
    r.initialize(0)
    frames = {}
    for tr in ("rccl", "copy"):
        if scheme == "bands":
            g = ShardedGroup(r, world, replicated=True)
            g.initialize([0] * world, tr)
        else:
            g = ShardedGroup(r, world)
            g.initialize([0] * world, tr)
            g.set_scheme(scheme)
        assert g.transport == tr, (g.transport, tr)
        frames[tr] = [g.render_host(V, P, W, H) for V, P in orbit_views(W, H, 2)]
        g.close()
    for (V, P), a, b in zip(orbit_views(W, H, 2), frames["rccl"], frames["copy"]):
        nd = int(np.count_nonzero(a.view(np.uint32) != b.view(np.uint32)))
        assert nd == 0, (world, scheme, "rccl vs copy", nd)
        if scheme != "slabs":  # rows and bands: the 1-GPU frame
            ref = r.render_host(V, P, W, H)
            assert int(np.count_nonzero(a.view(np.uint32) != ref.view(np.uint32))) == 0, (world, scheme, "vs 1 GPU")
    print("ok", world, scheme, mode, sh)

run(2, "rows", "tile", 3, 640, 400, 60000, 111)
run(3, "rows", "live50", 0, 960, 540, 80000, 112)
run(2, "slabs", "tile", 0, 640, 400, 60000, 113)
run(3, "slabs", "live50", 3, 640, 400, 60000, 114)
run(2, "bands", "tile", 3, 640, 400, 60000, 115)
"""


def test_group_rccl_stub_bitexact(built):
    """The group's RCCL transport (grouped ncclSend/ncclRecv all-to-all and
    band gather, ncclAllReduce / ncclAllGather / ncclReduce of the slab
    scheme) on a one-GPU box: GS_RCCL_LIB points the group's dlopen at the
    test stub (tests/cpp/rccl_stub.hip: the same entry points as
    stream-ordered peer copies, ranks sharing device 0).  Every frame equals
    the copy transport's bit for bit, and rows and bands the 1-GPU frame.
    Its own process: RCCL is resolved once per process."""
    import os
    import subprocess
    import sys
    from pathlib import Path

    from gaussian_splat_amd.build import RCCL_STUB
    root = Path(__file__).resolve().parents[1]
    assert RCCL_STUB.exists(), "build() makes tests/cpp/librccl_stub.so"
    env = dict(os.environ, GS_RCCL_LIB=str(RCCL_STUB))
    p = subprocess.run([sys.executable, "-c", _STUB_SCRIPT, str(root)], env=env, capture_output=True, text=True,
                       timeout=170)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert p.stdout.count("ok ") == 5, p.stdout


_REAL_RCCL_SCRIPT = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
sys.path.insert(0, sys.argv[1] + "/tests")
from conftest import orbit_views
from gaussian_splat_amd import InstancedSplatRenderer, Options, ShardedGroup
from gaussian_splat_amd import scene as S

W, H = 640, 400
sc = S.activate(S.synthetic_raw(60000, seed=116, aspect=W / H, rest=True), 3)
r = InstancedSplatRenderer(sc, Options(sh_degree=3, crop=False))
r.initialize(0)
for scheme in ("rows", "bands"):
    g = ShardedGroup(r, 1, replicated=scheme == "bands")
    g.initialize([0], "rccl")
    assert g.transport == "rccl", g.transport
    if scheme == "rows":
        g.set_scheme("rows")
    for V, P in orbit_views(W, H, 2):
        a, ref = g.render_host(V, P, W, H), r.render_host(V, P, W, H)
        assert int(np.count_nonzero(a.view(np.uint32) != ref.view(np.uint32))) == 0, scheme
    g.close()
    print("ok", scheme)
"""


def test_group_real_rccl_one_rank(built):
    """The group over the real RCCL library (the group's dlopen of librccl,
    ncclCommInitAll, the grouped ncclSend/ncclRecv of the record exchange and
    the band gather), with the one rank this box has (every record and band to
    itself; RCCL takes one device per rank, so two ranks need two GPUs):
    rows and bands frames equal the 1-GPU frame bit for bit.  Its own process,
    GS_RCCL_LIB unset: RCCL is resolved once per process."""
    import os
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k != "GS_RCCL_LIB"}
    p = subprocess.run([sys.executable, "-c", _REAL_RCCL_SCRIPT, str(root)], env=env, capture_output=True, text=True,
                       timeout=170)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert p.stdout.count("ok ") == 2, p.stdout


def test_group_bounded_wait(built):
    """Every host wait of a group is bounded (gs_group_set_timeout): a wait
    that cannot finish in time fails the frame with GS_ERR_COMM and leaves
    the group unusable, instead of hanging.  Here a 4K host-output frame of
    a 6M-splat scene (tens of ms) under a 1 ms bound."""
    from gaussian_splat_amd import GsError, InstancedSplatRenderer, Options, ShardedGroup
    W, H = 3840, 2160
    sc = _scene(2_000_000, 91, 0, W / H)
    r = InstancedSplatRenderer(sc, Options(crop=False))
    r.initialize(0)
    g = _group(r, 2)
    V, P = orbit_views(W, H, 1)[0]
    ref = r.render_host(V, P, W, H)
    np.testing.assert_array_equal(g.render_host(V, P, W, H).view(np.uint32), ref.view(np.uint32))
    with pytest.raises(GsError):
        g.set_timeout(0)
    g.set_timeout(1)
    # host output into pinned memory: the 133-MB device-to-host copy alone
    # (asynchronous into pinned memory) outlasts a 1 ms bound
    import ctypes as C
    import torch
    from gaussian_splat_amd._lib import lib
    from gaussian_splat_amd.api import _mat16
    pinned = torch.empty((H, W, 4), dtype=torch.float32, pin_memory=True)
    rc = lib().gs_group_render(g._g, _mat16(V), _mat16(P), W, H, C.c_void_p(pinned.data_ptr()), 0, None)
    assert rc == 6, rc  # GS_ERR_COMM: the wait expired
    with pytest.raises(GsError, match="unusable"):
        g.render_host(V, P, W, H)
    torch.cuda.synchronize()  # the abandoned frame's work drains before the buffers go


def test_group_rejects_rccl_on_shared_device(built):
    from gaussian_splat_amd import GsError, InstancedSplatRenderer, Options, ShardedGroup
    sc = _scene(1000, 5, 0, 1.0)
    r = InstancedSplatRenderer(sc, Options(crop=False))
    g = ShardedGroup(r, 2)
    with pytest.raises(GsError):
        g.initialize([0, 0], "rccl")


@pytest.mark.parametrize("world,mode,sh", [(2, "tile", 3), (4, "live50", 0)])
def test_group_replicated_bands_bitexact(built, world, mode, sh):
    """gs_create_replicated: the whole scene on every rank, owned rows per
    rank (GS_SCHEME_BANDS), gathered into the frame: the 1-GPU frame."""
    from gaussian_splat_amd import InstancedSplatRenderer, Options, ShardedGroup
    W, H = 960, 540
    sc = _scene(80000, 101 + world, sh, W / H)
    r = InstancedSplatRenderer(sc, Options(mode=mode, sh_degree=sh, crop=False))
    r.initialize(0)
    g = ShardedGroup(r, world, replicated=True)
    g.initialize([0] * world, "copy")
    for V, P in orbit_views(W, H, 2):
        ref = r.render_host(V, P, W, H)
        np.testing.assert_array_equal(g.render_host(V, P, W, H).view(np.uint32), ref.view(np.uint32))
    from gaussian_splat_amd import GsError
    with pytest.raises(GsError):
        g.set_scheme("rows")  # a replicated group renders bands only


def _pipelined_frames(g, views, W, H, host):
    """Pipelined group frames over a camera path: frame i comes back from call
    i + 1 (the last from flush)."""
    got = [g.render_pipelined(V, P, W, H, host=host) for V, P in views]
    assert got[0] is None, "the first pipelined call has no frame to return"
    got = got[1:] + [g.flush(W, H, host=host)]
    assert g.flush(W, H, host=host) is None  # (nothing left in flight)
    if not host:
        import torch
        torch.cuda.synchronize()
        got = [x.cpu().numpy() for x in got]
    return got


@pytest.mark.parametrize("world,mode,sh,host", [(2, "tile", 3, False), (3, "live50", 0, True), (4, "tile", 3, False)])
def test_group_rows_pipelined_bitexact(built, world, mode, sh, host):
    """Two frames in flight (gs_group_render_pipelined): frame k's record
    all-to-all on the ranks' exchange streams under frame k-1's render and
    gather; every frame comes back one call late, bit for bit the 1-GPU frame
    of its view, over a camera path with a resolution change in it."""
    from gaussian_splat_amd import GsError, InstancedSplatRenderer, Options
    W, H = 960, 540
    sc = _scene(120000, 141 + world, sh, W / H)
    r = InstancedSplatRenderer(sc, Options(mode=mode, sh_degree=sh, crop=False))
    r.initialize(0)
    g = _group(r, world)
    g.set_frames_in_flight(2)
    views = orbit_views(W, H, 4)
    frames = _pipelined_frames(g, views, W, H, host)
    for (V, P), got in zip(views, frames):
        ref = r.render_host(V, P, W, H)
        assert int(np.count_nonzero(got.view(np.uint32) != ref.view(np.uint32))) == 0
    # a resolution change between two frames in flight
    W2, H2 = 640, 400
    (V1, P1), (V2, P2) = orbit_views(W, H, 1)[0], orbit_views(W2, H2, 2)[1]
    assert g.render_pipelined(V1, P1, W, H, host=True) is None
    a = g.render_pipelined(V2, P2, W2, H2, host=True)
    with pytest.raises(GsError):
        g.render_host(V1, P1, W, H)  # (a frame is in flight)
    b = g.flush(W2, H2, host=True)
    np.testing.assert_array_equal(a.view(np.uint32), r.render_host(V1, P1, W, H).view(np.uint32))
    np.testing.assert_array_equal(b.view(np.uint32), r.render_host(V2, P2, W2, H2).view(np.uint32))
    # back to one frame at a time
    g.set_frames_in_flight(1)
    np.testing.assert_array_equal(g.render_host(V1, P1, W, H).view(np.uint32), r.render_host(V1, P1, W, H).view(np.uint32))


_STUB_PIPE_SCRIPT = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
sys.path.insert(0, sys.argv[1] + "/tests")
from conftest import orbit_views
from gaussian_splat_amd import InstancedSplatRenderer, Options, ShardedGroup
from gaussian_splat_amd import scene as S

def run(world, mode, sh, W, H, n, seed):
    sc = S.activate(S.synthetic_raw(n, seed=seed, aspect=W / H, rest=sh > 0), sh)
    r = InstancedSplatRenderer(sc, Options(mode=mode, sh_degree=sh, crop=False))
    r.initialize(0)
    views = orbit_views(W, H, 4)
    frames = {}
    for tr in ("rccl", "copy"):
        g = ShardedGroup(r, world)
        g.initialize([0] * world, tr)
        assert g.transport == tr, (g.transport, tr)
        g.set_frames_in_flight(2)
        got = [g.render_pipelined(V, P, W, H, host=True) for V, P in views]
        assert got[0] is None
        frames[tr] = got[1:] + [g.flush(W, H, host=True)]
        g.close()
    for (V, P), a, b in zip(views, frames["rccl"], frames["copy"]):
        ref = r.render_host(V, P, W, H)
        for tr, x in (("rccl", a), ("copy", b)):
            nd = int(np.count_nonzero(x.view(np.uint32) != ref.view(np.uint32)))
            assert nd == 0, (world, tr, "pipelined vs 1 GPU", nd)
    print("ok", world, mode, sh)

run(2, "tile", 3, 640, 400, 60000, 121)
run(3, "live50", 0, 960, 540, 80000, 122)
"""


def test_group_rccl_stub_pipelined_bitexact(built):
    """The pipelined rows scheme's RCCL branches (the exchange communicator
    set's grouped ncclSend/ncclRecv on the exchange streams, the band gather
    on the gather streams) on a one-GPU box through the test stub (as
    test_group_rccl_stub_bitexact): over a camera path every frame equals
    the 1-GPU frame bit for bit, for the RCCL and the copy transport."""
    import os
    import subprocess
    import sys
    from pathlib import Path

    from gaussian_splat_amd.build import RCCL_STUB
    root = Path(__file__).resolve().parents[1]
    assert RCCL_STUB.exists(), "build() makes tests/cpp/librccl_stub.so"
    env = dict(os.environ, GS_RCCL_LIB=str(RCCL_STUB))
    p = subprocess.run([sys.executable, "-c", _STUB_PIPE_SCRIPT, str(root)], env=env, capture_output=True, text=True,
                       timeout=170)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert p.stdout.count("ok ") == 2, p.stdout
