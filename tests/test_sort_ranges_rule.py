"""The sort's run-end merge skip (radix_sort.hip, rts_pass_kernel, rflag), restated in numpy.

The last LSD pass of the bin sort records each bin's extent in the sorted pairs
(``ranges``, read by the per-bin depth sort and the composite) with atomicMin
merges at every run end a tile sees. A tile skips the merges its neighbour tile
proves redundant: the neighbour lies wholly inside the tile's first (last) low
value and holds the digit. This test replays that rule tile by tile over random,
clustered, geometric and presorted keys and checks the merged extents against
the true runs of a stable sort. The kernel itself is checked bit-exactly on the
GPU by every frame test (the ranges feed every bin list).
"""
import numpy as np
import pytest

def sim(keys, shift, width, TILE):
    """One LSD pass over the high digit of keys already sorted by their low `shift` bits; returns merges made."""
    bits = shift + width; rmask = (1 << bits) - 1; lm = (1 << shift) - 1; mask = (1 << width) - 1
    x = keys[np.argsort(keys & lm, kind='stable')]  # pass-0 output (LSD)
    n = len(x); nt = (n + TILE - 1) // TILE
    d = (x >> shift) & mask
    C = np.zeros((mask + 1, nt), np.int64)
    for t in range(nt): C[:, t] = np.bincount(d[t*TILE:(t+1)*TILE], minlength=mask + 1)
    tot = C.sum(1); Cs = np.cumsum(C, 1) - C  # exclusive
    dstart = np.cumsum(tot) - tot
    out = x[np.argsort(d, kind='stable')]
    lo = np.full(rmask + 1, 2**32 - 1, np.int64); hi = np.full(rmask + 1, -1, np.int64); merges = 0
    for t in range(nt):
        t0, t1 = t*TILE, min(t*TILE + TILE, n)
        seg = x[t0:t1]; o = seg[np.argsort((seg >> shift) & mask, kind='stable')]
        lf, ll = seg[0] & lm, seg[-1] & lm
        fl = np.zeros(mask + 1, int)
        for dd in range(mask + 1):
            if t > 0 and (x[t0 - TILE] & lm) == lf and (x[t0 - 1] & lm) == lf and Cs[dd, t] != Cs[dd, t - 1]: fl[dd] |= 1
            if t1 < n:
                t2 = min(t1 + TILE, n)
                after = Cs[dd, t + 2] if t + 2 < nt else tot[dd]
                if (x[t1] & lm) == ll and (x[t2 - 1] & lm) == ll and after != Cs[dd, t + 1]: fl[dd] |= 2
        for j in range(len(o)):
            k = o[j]; rk = k & rmask; dd = (k >> shift) & mask
            g = dstart[dd] + Cs[dd, t] + (j - np.searchsorted((o >> shift) & mask, dd))
            assert out[g] == k
            s0 = j == 0 or (o[j-1] & rmask) != rk; s1 = j + 1 == len(o) or (o[j+1] & rmask) != rk
            l = k & lm
            if s0 and not (l == lf and fl[dd] & 1): lo[rk] = min(lo[rk], g); merges += 1
            if s1 and not (l == ll and fl[dd] & 2): hi[rk] = max(hi[rk], g + 1); merges += 1
    b = out & rmask
    for r in range(rmask + 1):
        w = np.nonzero(b == r)[0]
        if len(w): assert lo[r] == w[0] and hi[r] == w[-1] + 1, (r, lo[r], hi[r], w[0], w[-1])
        else: assert lo[r] == 2**32 - 1 and hi[r] == -1
    return merges


@pytest.mark.parametrize("trial", range(24))
def test_merge_skip_rule_gives_true_ranges(trial):
    rng = np.random.default_rng(1000 + trial)
    shift = int(rng.integers(1, 5))
    width = int(rng.integers(1, 5))
    tile = int(rng.choice([16, 64, 100]))
    n = int(rng.integers(1, 1500))
    nb = 1 << (shift + width)
    kind = trial % 4
    if kind == 0:  # uniform bins
        k = rng.integers(0, nb, n)
    elif kind == 1:  # three hot bins
        k = rng.choice(rng.integers(0, nb, 3), n)
    elif kind == 2:  # geometric: many tiles per low value, empty digits
        k = np.minimum(rng.geometric(0.05, n), nb - 1)
    else:  # already sorted
        k = np.sort(rng.integers(0, nb, n))
    k = (k | (rng.integers(0, 64, n) << (shift + width))).astype(np.int64)  # depth bits ride above
    sim(k, shift, width, tile)
