"""Multi-GPU rendering: splat-index shards, bin-row ownership, RCCL exchange.

DESIGN.md §6.  One process per GPU.  Rank r holds a contiguous splat-index
range of the scene.  Every 32-pixel bin row has one owning rank; by default
(`row_owner`) rank r owns a contiguous, balanced range of rows, so few splats
straddle an ownership boundary.  Per frame:

  1. gs_shard_project   project the local shard and pack a 48-B exchange
                        record for every (visible splat, owning rank) pair,
                        grouped by destination, index order inside
  2. all_to_all         exchange counts, then records (RCCL over xGMI)
  3. gs_shard_render    bin/sort/composite the received records into the
                        owned bin rows (a compact band buffer)
  4. gather             bands -> rank 0, scattered back into the frame

Pipelined (`ShardedRenderer(pipeline=True)`, two frames in flight): a call
projects frame k and starts its record exchange (asynchronous, on its own
process group), then renders and gathers frame k-1, whose records arrived
while frame k was projected; `flush()` finishes the last frame.  The link
transfer of one frame overlaps the other frame's compute.

Records arrive in source-rank order = global splat-index order, so each
owned bin sees exactly the single-GPU list order: the assembled frame is
bit-identical to a 1-GPU render (tests/test_gpu_parity.py,
tests/test_distributed.py).  The backend object does the per-rank compute:
`HipShardBackend` (libgsplat.so) in production; the gloo tests plug in a
CPU backend from tests/.

`BandRenderer` is SURVEY §8(e)'s fallback: every rank holds the whole
scene and renders only its owned bin rows (gs_band_render), then the bands
are gathered as above; no exchange, bit-identical like the row scheme.

`SlabRenderer` is the north star's literal scheme: rank d
composites depth slab d of the whole frame, then an RCCL reduce sums the
per-pixel RGBA + weight (alpha) contributions:

  1. gs_slab_project    preprocess; pair-weighted 15-bit depth-key histogram
  2. all_reduce         histogram (SUM) -> slab bounds of equal pair counts
  3. gs_slab_pack       one exchange record per visible splat, to its slab
  4. all_to_all         counts, then records
  5. gs_slab_render     the slab's bin lists + its own transmittance
  6. all_gather         transmittance of every slab
  7. gs_slab_composite  colour pass from the product of the farther slabs'
  8. reduce             SUM of the (C, delta alpha) contributions -> rank 0
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from . import _lib as L
from .api import InstancedSplatRenderer, Options, Scene, _mat16
from ._lib import check, lib

ROW = 32  # ownership unit: one 32-pixel bin row

# Bound of every rendezvous and collective of a rank (SURVEY §5 failure
# detection): a peer that never joins or stops answering makes the others
# raise within this time instead of hanging (the reference, one Metal
# device, has no such path: instanced_splat_renderer.mm:319-336).
DEFAULT_TIMEOUT_S = 120.0


def init_ranks(backend: str = "nccl", timeout_s: float = DEFAULT_TIMEOUT_S, device=None, **kw):
    """torch.distributed.init_process_group with a bounded timeout: the
    rendezvous and every later collective of the group (gloo: each
    send/recv; nccl = RCCL: the watchdog with async error handling, which
    aborts the communicator) fail after timeout_s.  `kw`: init_method, rank,
    world_size (default: the torchrun environment)."""
    import datetime
    import os

    import torch.distributed as dist

    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    td = datetime.timedelta(seconds=float(timeout_s))
    if backend == "nccl" and device is not None:
        kw["device_id"] = device
    dist.init_process_group(backend, timeout=td, **kw)


def row_owner(height: int, world: int) -> np.ndarray:
    """Default owner table (the C-ABI's, gs_shard_set_rows): rank r owns the
    contiguous bin rows [r*R/world, (r+1)*R/world), R = ceil(height/32)."""
    R = (height + ROW - 1) // ROW
    o = np.zeros(R, np.uint8)
    for r in range(world):
        o[r * R // world:(r + 1) * R // world] = r
    return o


def band_rows(height: int, world: int, owner=None) -> int:
    """Pixel rows of the (padded, equal-size) band buffer of every rank."""
    o = row_owner(height, world) if owner is None else np.asarray(owner)
    return int(max((o == r).sum() for r in range(world))) * ROW


def assemble(bands, width: int, height: int, world: int, owner=None):
    """Scatter the rank bands (owned rows stacked in ascending order) into a frame."""
    import torch

    o = row_owner(height, world) if owner is None else np.asarray(owner)
    R = len(o)
    frame = torch.zeros((R * ROW, width, 4), dtype=torch.float32, device=bands[0].device)
    for r, b in enumerate(bands):
        rows = np.nonzero(o == r)[0]
        if len(rows) == 0:
            continue
        src = b.view(-1, ROW, width, 4)[: len(rows)]
        starts = rows.tolist()
        # contiguous runs of owned rows copy as one block
        k = 0
        while k < len(starts):
            e = k
            while e + 1 < len(starts) and starts[e + 1] == starts[e] + 1:
                e += 1
            frame[starts[k] * ROW:(starts[e] + 1) * ROW] = src[k:e + 1].reshape(-1, width, 4)
            k = e + 1
    return frame[:height]


def gather_frame(band, width: int, height: int, world: int, rank: int, owner=None, group=None, p2p=None,
                 pending=None):
    """The rank bands -> the full frame on rank 0 (None elsewhere).  With the
    default contiguous ownership over RCCL every rank sends its valid rows
    straight into their place in rank 0's frame (point-to-point, no padded
    bands, no reassembly copies); gloo (host-staged) and custom owner tables
    gather the padded bands and scatter them (`assemble`).  p2p=True forces the
    point-to-point path (CPU tensors over gloo: its test).
    pending (a list; point-to-point path only): the transfers are left in
    flight and their works appended to it, so the caller's stream is not made
    to wait for them (ShardedRenderer's pipelined frames wait on the user's
    stream, not on the compute stream)."""
    import torch
    import torch.distributed as dist

    if p2p is None:
        p2p = owner is None and not _host_staged(group)
    if p2p:
        assert owner is None, "point-to-point gather: contiguous default ownership only"
        R = (height + ROW - 1) // ROW
        spans = [(min(height, r * R // world * ROW), min(height, (r + 1) * R // world * ROW)) for r in range(world)]
        if rank == 0:
            frame = torch.empty((height, width, 4), dtype=torch.float32, device=band.device)
            ops = [dist.P2POp(dist.irecv, frame[y0:y1], r, group) for r, (y0, y1) in enumerate(spans)
                   if r > 0 and y1 > y0]
            reqs = dist.batch_isend_irecv(ops) if ops else []
            y0, y1 = spans[0]
            if y1 > y0:
                frame[y0:y1].copy_(band[: y1 - y0])
            if pending is not None:
                pending.extend(reqs)
            else:
                for q in reqs:
                    q.wait()
            return frame
        y0, y1 = spans[rank]
        if y1 > y0:
            # (a batch of one, as rank 0's receives: every rank of the group
            # enters its first point-to-point call through the same API, as
            # torch.distributed asks of RCCL/NCCL)
            reqs = dist.batch_isend_irecv([dist.P2POp(dist.isend, band[: y1 - y0], 0, group)])
            if pending is not None:
                pending.extend(reqs)
            else:
                for q in reqs:
                    q.wait()
        return None
    if _host_staged(group):
        hb = band.cpu()
        bands = [hb.new_empty(hb.shape) for _ in range(world)] if rank == 0 else None
        dist.gather(hb, bands, dst=0, group=group)
        bands = [b.to(band.device) for b in bands] if rank == 0 else None
    else:
        bands = [band.new_empty(band.shape) for _ in range(world)] if rank == 0 else None
        dist.gather(band, bands, dst=0, group=group)
    return assemble(bands, width, height, world, owner) if rank == 0 else None


class HipShardBackend:
    """Per-rank compute through libgsplat.so (device buffers are torch tensors)."""

    def __init__(self, shard: Scene, rank: int, world: int, index_base: int, options: Options, device: int,
                 owner=None):
        import torch

        self.r = InstancedSplatRenderer(shard, options)
        self.r.initialize(device)
        check(lib().gs_shard_configure(self.r._h, rank, world, index_base), "gs_shard_configure")
        self.owner = None if owner is None else np.ascontiguousarray(owner, np.uint8)
        if self.owner is not None:  # same table on every rank (default: contiguous ranges)
            check(lib().gs_shard_set_rows(self.r._h, self.owner.ctypes.data, len(self.owner)),
                  "gs_shard_set_rows")
        self.world, self.rank, self.device = world, rank, torch.device(f"cuda:{device}")
        self.xbytes = int(lib().gs_exchange_record_bytes())
        self.xregions = exchange_regions()
        self._send = [torch.empty(max(1, shard.n * world * self.xbytes), dtype=torch.uint8, device=self.device)]

    @property
    def send(self):
        return self._send[0]

    def project(self, view, proj, width, height, slot: int = 0):
        """Project and pack into send buffer `slot` (0/1: a pipelined frame's
        exchange may still be reading the other)."""
        import torch

        while len(self._send) <= slot:
            self._send.append(torch.empty_like(self._send[0]))
        buf = self._send[slot]
        counts = (C.c_int64 * self.world)()
        stream = torch.cuda.current_stream(self.device).cuda_stream
        check(lib().gs_shard_project(self.r._h, _mat16(view), _mat16(proj), width, height,
                                     C.c_void_p(buf.data_ptr()), buf.numel(), counts,
                                     C.c_void_p(stream)), "gs_shard_project")
        return buf, [int(c) for c in counts]

    def empty(self, nbytes):
        import torch

        return torch.empty(max(1, nbytes), dtype=torch.uint8, device=self.device)

    def render(self, recv, nrec, width, height, composite_stream=None):
        """The band of the received records.  composite_stream (a torch
        stream): the lists on the current stream, the composite there
        (gs_shard_render_split), so the next projection on the current stream
        runs beside it; the band is then complete on composite_stream."""
        import torch

        band = torch.empty((band_rows(height, self.world, self.owner), width, 4), dtype=torch.float32,
                           device=self.device)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        if composite_stream is not None:
            check(lib().gs_shard_render_split(self.r._h, C.c_void_p(recv.data_ptr()), int(nrec), width, height,
                                              C.c_void_p(band.data_ptr()), C.c_void_p(stream),
                                              C.c_void_p(composite_stream.cuda_stream)), "gs_shard_render_split")
            if recv.is_cuda:
                recv.record_stream(composite_stream)  # (read by the composite)
            band.record_stream(composite_stream)
        else:
            check(lib().gs_shard_render(self.r._h, C.c_void_p(recv.data_ptr()), int(nrec), width, height,
                                        C.c_void_p(band.data_ptr()), C.c_void_p(stream)), "gs_shard_render")
        return band


class HipBandBackend:
    """Per-rank compute of the replicated-scene band scheme (SURVEY §8(e)
    fallback): the rank holds the WHOLE scene and renders its
    owned bin rows (gs_band_render); no exchange."""

    def __init__(self, scene: Scene, rank: int, world: int, options: Options, device: int, owner=None):
        import torch

        self.r = InstancedSplatRenderer(scene, options)
        self.r.initialize(device)
        check(lib().gs_shard_configure(self.r._h, rank, world, 0), "gs_shard_configure")
        self.owner = None if owner is None else np.ascontiguousarray(owner, np.uint8)
        if self.owner is not None:
            check(lib().gs_shard_set_rows(self.r._h, self.owner.ctypes.data, len(self.owner)), "gs_shard_set_rows")
        self.world, self.rank, self.device = world, rank, torch.device(f"cuda:{device}")

    def render(self, view, proj, width, height):
        import torch

        rows = height if self.world == 1 else band_rows(height, self.world, self.owner)
        band = torch.empty((rows, width, 4), dtype=torch.float32, device=self.device)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        check(lib().gs_band_render(self.r._h, _mat16(view), _mat16(proj), width, height,
                                   C.c_void_p(band.data_ptr()), C.c_void_p(stream)), "gs_band_render")
        return band


class BandRenderer:
    """One rank of a replicated-scene band frame (torch.distributed initialised)."""

    def __init__(self, backend, rank: int, world: int, group=None):
        self.b, self.rank, self.world, self.group = backend, rank, world, group

    def render(self, view, proj, width, height, gather: bool = True):
        """The full frame on rank 0 (None elsewhere) when gather=True, else
        this rank's band."""
        band = self.b.render(view, proj, width, height)
        if not gather:
            return band
        if self.world == 1:
            return band[:height]
        return gather_frame(band, width, height, self.world, self.rank, self.b.owner, self.group)


SLAB_BINS = 2048      # GS_SLAB_BINS: slab histogram bins ...
SLAB_BIN_KEYS = 16    # ... of 16 15-bit depth keys


def slab_bounds(hist, world: int) -> np.ndarray:
    """Slab key bounds [world + 1] of equal pair counts from the summed
    histogram (gs_slab_bounds, host code of libgsplat.so)."""
    h = np.ascontiguousarray(np.asarray(hist).view(np.uint64) if np.asarray(hist).dtype == np.int64
                             else np.asarray(hist, np.uint64))
    assert h.shape == (SLAB_BINS,)
    b = np.zeros(world + 1, np.uint32)
    check(lib().gs_slab_bounds(h.ctypes.data, int(world), b.ctypes.data), "gs_slab_bounds")
    return b


class HipSlabBackend(HipShardBackend):
    """Per-rank compute of the depth-slab scheme through libgsplat.so."""

    def project(self, view, proj, width, height):
        import torch

        hist = torch.empty(SLAB_BINS, dtype=torch.int64, device=self.device)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        check(lib().gs_slab_project(self.r._h, _mat16(view), _mat16(proj), width, height,
                                    C.c_void_p(hist.data_ptr()), C.c_void_p(stream)), "gs_slab_project")
        return hist

    def pack(self, bounds):
        import torch

        b = np.ascontiguousarray(bounds, np.uint32)
        counts = (C.c_int64 * self.world)()
        stream = torch.cuda.current_stream(self.device).cuda_stream
        check(lib().gs_slab_pack(self.r._h, b.ctypes.data, C.c_void_p(self.send.data_ptr()), self.send.numel(),
                                 counts, C.c_void_p(stream)), "gs_slab_pack")
        return self.send, [int(c) for c in counts]

    def render(self, recv, nrec, width, height):
        import torch

        self._recv = recv  # the colour pass reads the records again
        t = torch.empty((height, width), dtype=torch.float32, device=self.device)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        check(lib().gs_slab_render(self.r._h, C.c_void_p(recv.data_ptr()), int(nrec), width, height,
                                   C.c_void_p(t.data_ptr()), C.c_void_p(stream)), "gs_slab_render")
        return t

    def composite(self, t_all):
        import torch

        h, w = t_all.shape[1], t_all.shape[2]
        out = torch.empty((h, w, 4), dtype=torch.float32, device=self.device)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        check(lib().gs_slab_composite(self.r._h, C.c_void_p(t_all.data_ptr()), C.c_void_p(out.data_ptr()),
                                      C.c_void_p(stream)), "gs_slab_composite")
        self._recv = None
        return out


def shard_bounds(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous index range of rank `rank` (balanced)."""
    b = n * rank // world
    e = n * (rank + 1) // world
    return b, e


def _host_staged(group) -> bool:
    """gloo moves host tensors only: stage device buffers through host memory
    (a rehearsal path; RCCL/nccl exchanges device memory directly)."""
    import torch.distributed as dist

    return dist.get_backend(group) == "gloo"


def exchange_regions() -> tuple:
    """Bytes per record of each exchange region (gs_exchange_regions): the
    48-B records, then the rect lo / hi words and depth keys (gsplat.h)."""
    n = int(lib().gs_exchange_regions(None))
    b = (C.c_int32 * n)()
    lib().gs_exchange_regions(b)
    return tuple(int(x) for x in b)


def region_views(buf, total: int, regions):
    """The regions of an exchange buffer holding `total` records."""
    out, o = [], 0
    for b in regions:
        out.append(buf[o: o + total * b])
        o += total * b
    return out


class PendingExchange:
    """A record all_to_all in flight (exchange_start); wait() -> (recv, nrec)."""

    def __init__(self, works, recv, total, dev):
        self.works, self.recv, self.total, self.dev = works, recv, total, dev

    def wait(self):
        for w in self.works:
            w.wait()  # (RCCL: the current stream waits for the exchange)
        self.works = []
        recv = self.recv if self.recv.device == self.dev else self.recv.to(self.dev)
        return recv, self.total


def exchange_start(send, counts, regions, world, group=None) -> PendingExchange:
    """all_to_all of counts (the host sizes the receive buffer), then one
    all_to_all per exchange region (records, rect lo, rect hi, depth keys;
    `regions` = their bytes per record), started asynchronously."""
    import torch
    import torch.distributed as dist

    regions = (regions,) if isinstance(regions, int) else tuple(regions)
    xb = sum(regions)
    dev = send.device
    cdev = torch.device("cpu") if _host_staged(group) else dev
    sc = torch.tensor(counts, dtype=torch.int64, device=cdev)
    rc = torch.empty(world, dtype=torch.int64, device=cdev)
    dist.all_to_all_single(rc, sc, group=group)
    rcounts = [int(x) for x in rc.cpu().tolist()]
    total, sent = sum(rcounts), sum(counts)
    recv = torch.empty(max(1, total * xb), dtype=torch.uint8, device=cdev)
    src = send[: sent * xb] if cdev == dev else send[: sent * xb].cpu()
    works = [dist.all_to_all_single(r, q, [c * b for c in rcounts], [c * b for c in counts], group=group,
                                    async_op=True)
             for b, r, q in zip(regions, region_views(recv, total, regions), region_views(src, sent, regions))]
    return PendingExchange(works, recv, total, dev)


def exchange(send, counts, regions, world, group=None):
    """all_to_all of counts then of the record regions; returns (recv, nrec)."""
    return exchange_start(send, counts, regions, world, group).wait()


def virtual_exchange(sends, regions, world: int):
    """The all_to_all by slicing (every rank in one process): for each
    destination its received buffer (region by region, source-rank order
    inside) and record count, from every source's (send, counts)."""
    import torch

    regions = (regions,) if isinstance(regions, int) else tuple(regions)
    out = []
    for dst in range(world):
        parts, nrec = [], 0
        views = [region_views(buf, sum(counts), regions) for buf, counts in sends]
        for k, b in enumerate(regions):
            for src in range(world):
                counts = sends[src][1]
                off = sum(counts[:dst]) * b
                parts.append(views[src][k][off: off + counts[dst] * b])
        nrec = sum(sends[src][1][dst] for src in range(world))
        out.append((torch.cat(parts) if nrec else None, nrec))
    return out


class ShardedRenderer:
    """One rank of a multi-GPU frame (torch.distributed must be initialised).

    pipeline=True: two frames in flight.  render() projects this frame and
    starts its record exchange on `exchange_group` (its own communicator, so
    it runs beside the gather), then renders and gathers the PREVIOUS frame
    and returns it (None on the first call); flush() finishes the frame still
    in flight.  Every rank must make the same calls.  Over RCCL a pipelined
    rank computes on its own stream: the band transfers of the gather are
    waited for by the caller's stream only (rank 0's frame is ready there), so
    the next frame's projection does not queue behind them.  Per call the
    rank's stream runs projection k+1 then render k; the host exchanges frame
    k+1's counts while the GPU renders k, and the record exchange of k+1
    starts from a stream that waited for its projection alone."""

    def __init__(self, backend, rank: int, world: int, group=None, pipeline: bool = False, exchange_group=None,
                 own_stream: Optional[bool] = None):
        import torch

        self.b, self.rank, self.world, self.group = backend, rank, world, group
        self.pipeline = pipeline
        self.xgroup = exchange_group if exchange_group is not None else group
        self._pending = None
        self._slot = 0
        dev = getattr(backend, "device", None)
        # own_stream: None = over RCCL only (gloo stages through the host,
        # which waits anyway); True also over gloo (its test on one GPU)
        if own_stream is None:
            own_stream = not _host_staged(group)
        self._cs = (torch.cuda.Stream(dev) if pipeline and own_stream and world > 1 and dev is not None
                    and dev.type == "cuda" else None)
        # the next frame's exchange is issued from a stream that waited only
        # for its projection, so it does not queue behind this frame's render
        self._xs = torch.cuda.Stream(dev) if self._cs is not None else None
        # the render's composite (and the gather behind it) on a stream of its
        # own, so the next projection runs beside it (gs_shard_render_split;
        # GS_ROWS_SPLIT=0: one stream, A/B)
        import os

        split = os.environ.get("GS_ROWS_SPLIT", "1") != "0" and getattr(type(backend), "render", None) is HipShardBackend.render
        self._ccs = torch.cuda.Stream(dev) if self._cs is not None and split else None
        self._inflight = []  # (band, frame) of the last gather, alive until the next frame

    def _finish(self, pend, width, height, gather, works=None):
        recv, nrec = pend.wait()
        return self._gather(self.b.render(recv, nrec, width, height), width, height, gather, works)

    def _gather(self, band, width, height, gather, works=None):
        if not gather:
            return band
        if self.world == 1:
            return assemble([band], width, height, 1)
        out = gather_frame(band, width, height, self.world, self.rank, getattr(self.b, "owner", None), self.group,
                           pending=works)
        if works is not None:
            self._inflight.append((band, out))  # (alive until their transfers are done)
        return out

    def render(self, view, proj, width, height, gather: bool = True):
        """Returns the full frame on rank 0 (None elsewhere) when gather=True,
        else this rank's band buffer (pipelined: the previous frame's)."""
        if not self.pipeline:
            send, counts = self.b.project(view, proj, width, height)
            return self._finish(exchange_start(send, counts, self.b.xregions, self.world, self.group),
                                width, height, gather)
        if self._cs is None:
            return self._step(view, proj, width, height, gather, None)
        import torch

        # (the rank's stream does not wait for the caller's: nothing the frame
        # reads is written there, and the caller's stream holds the waits for
        # the previous gather, which this frame must not queue behind)
        user = torch.cuda.current_stream(self._cs.device)
        works = []
        with torch.cuda.stream(self._cs):
            out = self._step(view, proj, width, height, gather, works)
        return self._land(out, works, user)

    def _step(self, view, proj, width, height, gather, works):
        send, counts = self.b.project(view, proj, width, height, slot=self._slot)
        self._slot ^= 1
        if self._xs is None:
            nxt = (exchange_start(send, counts, self.b.xregions, self.world, self.xgroup), width, height, gather)
            old, self._inflight = self._inflight, []
            out = self._finish(*self._pending, works=works) if self._pending is not None else None
            del old  # (the previous gather's tensors: its transfers were waited for by the caller's stream)
            self._pending = nxt
            return out
        import torch

        # The rank's stream: the previous frame's render is queued right
        # behind this projection, before the host exchanges the counts (the
        # GPU renders meanwhile); the exchange starts from its own stream,
        # which waited for the projection alone; then the gather.
        projected = torch.cuda.Event()
        projected.record(self._cs)
        old, self._inflight = self._inflight, []
        band = None
        if self._pending is not None:
            pend, w_, h_, g_ = self._pending
            recv, nrec = pend.wait()
            band = self.b.render(recv, nrec, w_, h_, **({"composite_stream": self._ccs} if self._ccs else {}))
        with torch.cuda.stream(self._xs):
            self._xs.wait_event(projected)
            nxt = (exchange_start(send, counts, self.b.xregions, self.world, self.xgroup), width, height, gather)
        if nxt[0].recv.is_cuda:
            nxt[0].recv.record_stream(self._cs)  # (received on the exchange stream, read on the rank's)
        out = None
        if self._pending is not None:
            if self._ccs is not None:  # (the band is complete on the composite's stream: the gather starts there)
                with torch.cuda.stream(self._ccs):
                    out = self._gather(band, *self._pending[1:], works=works)
            else:
                out = self._gather(band, *self._pending[1:], works=works)
        del old  # (the previous gather's tensors: its transfers were waited for by the caller's stream)
        self._pending = nxt
        return out

    def _land(self, out, works, user):
        """The frame's compute (the rank's stream) and the gather's transfers,
        waited for by the caller's stream; the frame is marked in use there."""
        user.wait_stream(self._cs)
        if self._ccs is not None:
            user.wait_stream(self._ccs)
        for w in works:
            w.wait()
        if out is not None:
            out.record_stream(user)
        return out

    def flush(self):
        """The frame still in flight (pipelined), or None."""
        if self._pending is None:
            return None
        p, self._pending = self._pending, None
        if self._cs is None:
            return self._finish(*p)
        import torch

        user = torch.cuda.current_stream(self._cs.device)
        works = []
        with torch.cuda.stream(self._cs):
            out = self._finish(*p, works=works)
        return self._land(out, works, user)


def _all_reduce_sum(t, group):
    import torch.distributed as dist

    if _host_staged(group):
        h = t.cpu()
        dist.all_reduce(h, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, group=group)
    return t


def _all_gather(t, world, group):
    import torch
    import torch.distributed as dist

    if _host_staged(group):
        h = t.cpu()
        out = torch.empty((world,) + tuple(h.shape), dtype=h.dtype)
        dist.all_gather(list(out.unbind(0)), h, group=group)
        return out.to(t.device)
    out = torch.empty((world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t.contiguous(), group=group)
    return out


class SlabRenderer:
    """One rank of a depth-slab multi-GPU frame (torch.distributed initialised)."""

    def __init__(self, backend, rank: int, world: int, group=None):
        self.b, self.rank, self.world, self.group = backend, rank, world, group

    def render(self, view, proj, width, height, gather: bool = True):
        """The frame on rank 0 (None elsewhere) when gather=True (RGBA reduce),
        else this rank's (C, delta alpha) contribution."""
        import torch.distributed as dist

        hist = _all_reduce_sum(self.b.project(view, proj, width, height), self.group)
        bounds = slab_bounds(hist.cpu().numpy(), self.world)
        send, counts = self.b.pack(bounds)
        recv, nrec = exchange(send, counts, self.b.xregions, self.world, self.group)
        t = self.b.render(recv, nrec, width, height)
        t_all = _all_gather(t, self.world, self.group) if self.world > 1 else t[None]
        out = self.b.composite(t_all)
        if not gather or self.world == 1:
            return out
        if _host_staged(self.group):
            h = out.cpu()
            dist.reduce(h, dst=0, group=self.group)
            out.copy_(h)
        else:
            dist.reduce(out, dst=0, group=self.group)
        return out if self.rank == 0 else None


def render_virtual_slabs(scene: Scene, world: int, view, proj, width: int, height: int, sh_degree: int = 0,
                         mode: str = "tile", device: int = 0, parts: bool = False):
    """Depth-slab scheme with all ranks in one process on one GPU (collectives
    by slicing / summing in rank order).  Returns the frame, and with
    parts=True also the bounds, per-slab transmittance and contributions."""
    import torch

    opts = Options(mode=mode, sh_degree=sh_degree, crop=False)
    backends = []
    for r in range(world):
        b, e = shard_bounds(scene.n, world, r)
        be = HipSlabBackend(scene.subset(slice(b, e)), r, world, b, opts, device)
        backends.append(be)
    hist = sum(be.project(view, proj, width, height) for be in backends)
    bounds = slab_bounds(hist.cpu().numpy(), world)
    sends = [be.pack(bounds) for be in backends]
    ts, recvs = [], []
    for dst, (recv, nrec) in enumerate(virtual_exchange(sends, backends[0].xregions, world)):
        recvs.append(recv if nrec else backends[dst].empty(backends[dst].xbytes))
        ts.append(backends[dst].render(recvs[-1], nrec, width, height))
    t_all = torch.stack(ts)
    contrib = [be.composite(t_all) for be in backends]
    frame = contrib[0].clone()
    for c in contrib[1:]:
        frame += c
    torch.cuda.synchronize()
    if parts:
        return (frame.cpu().numpy(), bounds, t_all.cpu().numpy(), [c.cpu().numpy() for c in contrib],
                [r.cpu().numpy() for r in recvs])
    return frame.cpu().numpy()


class VirtualShards:
    """All `world` ranks of the row scheme in one process on one GPU, the
    exchange by slicing: the same kernels and record protocol as the
    multi-process path, frame after frame (so a rank's depth cuts carry over,
    DESIGN.md §6).  `options` as for InstancedSplatRenderer (crop off)."""

    def __init__(self, scene: Scene, world: int, options: Options, device: int = 0, owner=None):
        self.world, self.owner = world, owner
        self.backends = []
        for r in range(world):
            b, e = shard_bounds(scene.n, world, r)
            self.backends.append(HipShardBackend(scene.subset(slice(b, e)), r, world, b, options, device, owner))

    def set_rows(self, owner):
        """A new bin-row owner table on every rank (gs_shard_set_rows)."""
        o = np.ascontiguousarray(owner, np.uint8)
        for be in self.backends:
            be.owner = o
            check(lib().gs_shard_set_rows(be.r._h, o.ctypes.data, len(o)), "gs_shard_set_rows")
        self.owner = o

    def render(self, view, proj, width: int, height: int):
        """The assembled frame (device tensor, height x width x 4)."""
        import torch

        sends = [be.project(view, proj, width, height) for be in self.backends]
        bands = []
        for be, (recv, nrec) in zip(self.backends, virtual_exchange(sends, self.backends[0].xregions, self.world)):
            bands.append(be.render(recv if nrec else be.empty(be.xbytes), nrec, width, height))
        return assemble(bands, width, height, self.world, self.owner)


def render_virtual_shards(scene: Scene, world: int, view, proj, width: int, height: int, sh_degree: int = 0,
                          mode: str = "tile", device: int = 0, cap: int = 0, owner=None) -> np.ndarray:
    """One frame of VirtualShards (new ranks, so no depth cuts carried)."""
    import torch

    vs = VirtualShards(scene, world, Options(mode=mode, sh_degree=sh_degree, crop=False, cap=cap), device, owner)
    frame = vs.render(view, proj, width, height)
    torch.cuda.synchronize()
    return frame.cpu().numpy()
