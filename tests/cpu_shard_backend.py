"""CPU stand-in for HipShardBackend (test infrastructure).

Per-rank compute by the oracle; the exchange layout (gsplat.h: 48-B records,
then rect lo / hi words and depth keys, each region grouped by destination),
the destination rule (bin-row owner table) and the band layout are the
product's, so gloo runs of gaussian_splat_amd.distributed.ShardedRenderer
exercise the real exchange / gather / assembly protocol on CPU.
"""
import numpy as np

from oracle import oracle_py as O

XREC = O.RECORD_DTYPE  # 48-B exchange record: the projection's record
assert XREC.itemsize == 48
XREGIONS = (48, 4, 4, 4)


def _pack(parts):
    """Exchange regions of the per-destination (records, depth keys)."""
    import torch

    recs = np.concatenate([r for r, _ in parts]) if parts else np.zeros(0, XREC)
    keys = np.concatenate([k for _, k in parts]).astype(np.uint32) if parts else np.zeros(0, np.uint32)
    buf = np.concatenate([recs.view(np.uint8), recs["rect_lo"].astype(np.uint32).view(np.uint8),
                          recs["rect_hi"].astype(np.uint32).view(np.uint8), keys.view(np.uint8)])
    return torch.from_numpy(buf.copy() if buf.size else np.zeros(1, np.uint8))


def _unpack(recv, nrec):
    raw = recv.numpy()[: nrec * 60]
    rec = raw[: nrec * 48].copy().view(XREC)
    dkey = raw[nrec * 56: nrec * 60].copy().view(np.uint32)
    return rec, dkey


class OracleShardBackend:
    xbytes = 60
    xregions = XREGIONS

    def __init__(self, shard, rank, world, index_base, sh_degree=0, mode="tile", cap=0):
        self.shard, self.rank, self.world, self.base = shard, rank, world, index_base
        self.sh, self.mode, self.cap = sh_degree, mode, cap

    def project(self, view, proj, width, height, slot=0):
        from gaussian_splat_amd.distributed import row_owner

        rec, dk, nt = O.project(self.shard, view, proj, width, height, sh_degree=self.sh)
        vis = nt > 0
        owner = row_owner(height, self.world)
        ty0 = (rec["rect_lo"] >> 16) >> 5  # 32-px bin rows
        ty1 = (rec["rect_hi"] >> 16) >> 5
        w = self.world
        parts, counts = [], []
        for d in range(w):
            rows = np.nonzero(owner == d)[0]
            touch = np.zeros(len(nt), bool)
            if len(rows):  # a rank owns a contiguous range [rows[0], rows[-1]]
                touch = (ty0 <= rows[-1]) & (ty1 >= rows[0])
            idx = np.nonzero(vis & touch)[0]
            parts.append((rec[idx], dk[idx]))
            counts.append(len(idx))
        return _pack(parts), counts

    def render(self, recv, nrec, width, height):
        import torch

        rec, dkey = _unpack(recv, nrec)
        from gaussian_splat_amd.distributed import band_rows, row_owner

        band = np.zeros((band_rows(height, self.world), width, 4), np.float32)
        out = O.composite_records(rec, dkey, width, height, owner=row_owner(height, self.world),
                                  rank=self.rank, compact=True, mode=self.mode, cap=self.cap)
        band[: out.shape[0]] = out
        return torch.from_numpy(band)


class OracleSlabBackend(OracleShardBackend):
    """CPU stand-in for HipSlabBackend: depth slabs, oracle compute, the
    product's record format, slab rule (gs_slab_bounds) and collectives."""

    def project(self, view, proj, width, height):
        import torch

        from gaussian_splat_amd.distributed import SLAB_BIN_KEYS, SLAB_BINS

        self._rec, self._dk, self._nt = O.project(self.shard, view, proj, width, height, sh_degree=self.sh)
        vis = self._nt > 0
        hist = np.bincount(self._dk[vis] // SLAB_BIN_KEYS, weights=self._nt[vis], minlength=SLAB_BINS).astype(np.int64)
        return torch.from_numpy(hist)

    def pack(self, bounds):
        rec, dk, vis = self._rec, self._dk, self._nt > 0
        slab = np.searchsorted(np.asarray(bounds[1:-1], np.int64), dk.astype(np.int64), side="right")
        parts, counts = [], []
        for d in range(self.world):
            idx = np.nonzero(vis & (slab == d))[0]
            parts.append((rec[idx], dk[idx]))
            counts.append(len(idx))
        return _pack(parts), counts

    def render(self, recv, nrec, width, height):
        import torch

        self._srec, self._sdk = _unpack(recv, nrec)
        return torch.from_numpy(O.composite_slab(self._srec, self._sdk, width, height, 1, mode=self.mode))

    def composite(self, t_all):
        import torch

        ta = t_all.numpy()
        return torch.from_numpy(O.composite_slab(self._srec, self._sdk, ta.shape[2], ta.shape[1], 2, rank=self.rank,
                                                 t_all=ta, mode=self.mode))


class OracleBandBackend:
    """CPU stand-in for HipBandBackend: the whole scene on every rank, the
    rank's owned bin rows composited by the oracle into the product's band
    layout (no exchange)."""

    owner = None

    def __init__(self, scene, rank, world, sh_degree=0, mode="tile", cap=0):
        self.scene, self.rank, self.world = scene, rank, world
        self.sh, self.mode, self.cap = sh_degree, mode, cap

    def render(self, view, proj, width, height):
        import torch

        from gaussian_splat_amd.distributed import band_rows, row_owner

        rec, dk, nt = O.project(self.scene, view, proj, width, height, sh_degree=self.sh)
        vis = nt > 0
        band = np.zeros((band_rows(height, self.world), width, 4), np.float32)
        out = O.composite_records(rec[vis], dk[vis], width, height, owner=row_owner(height, self.world),
                                  rank=self.rank, compact=True, mode=self.mode, cap=self.cap)
        band[: out.shape[0]] = out
        return torch.from_numpy(band)
