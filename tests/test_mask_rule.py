"""The projection's exclusion-mask rule (preprocess.hip: ellipse_x,
cell_exclusion_mask, bins_from_cells, keep_one_bin), restated in float32
numpy and checked against brute force on random ellipses: a cell or bin is
excluded only when no pixel centre in it lies inside the q <= 2 ln 100
ellipse, and every non-empty rect keeps a bin.  (The device code itself is
held to this by the GPU frames: test_render_anisotropic_bitexact,
test_sorted_pairs_match_stable_sort.)"""
import math

import numpy as np

f = np.float32
QMAX = f(9.21034037197618)


def ellipse_x(ax, ay, bx, by):
    a = f(ax * ax + bx * bx); c = f(ay * ay + by * by); b = f(ax * ay + bx * by)
    cr = f(ax * by - ay * bx); det = f(cr * cr)
    ok = det > 0 and a > 0 and c > 0 and det < 3e38
    Q = f(QMAX * f(1.002) + f(1e-3))
    Qa = f(Q * a)
    e = dict(b=b, det=det, Qa=Qa, ok=ok)
    if ok:
        e["ia"] = f(1) / a
        idet = f(1) / det
        e["ymax"] = np.sqrt(f(Qa * idet)); e["xs"] = np.sqrt(f(Q * c * idet))
        e["ys"] = f(b * e["xs"] * (f(1) / c)); e["pad"] = f(0.01) + f(1e-3) * abs(e["xs"])
    return e


def cell_mask(e, cx, cy, x0, y0, x1, y1, shift):
    CS = 1 << shift
    cx0, cy0, cx1, cy1 = x0 >> shift, y0 >> shift, x1 >> shift, y1 >> shift
    if cx1 - cx0 >= 4 or cy1 - cy0 >= 4 or (cx1 == cx0 and cy1 == cy0) or not e["ok"]:
        return 0
    allb = (1 << (cx1 - cx0 + 1)) - 1
    excl = 0
    for r in range(cy1 - cy0 + 1):
        pyA = f((cy0 + r) * CS)
        yl = max(f(cy - (pyA + f(CS - 0.5))), -e["ymax"]); yh = min(f(cy - (pyA + f(0.5))), e["ymax"])
        keep = 0
        if yl <= yh:
            root = lambda y: np.sqrt(max(f(e["Qa"] - e["det"] * y * y), f(0)))
            rl, rh = root(yl), root(yh)
            b, ia, xs, ys, pad = e["b"], e["ia"], e["xs"], e["ys"], e["pad"]
            xmax = (xs if -ys >= yl and -ys <= yh else max(-b * yl + rl, -b * yh + rh) * ia) + pad
            xmin = (-xs if ys >= yl and ys <= yh else min(-b * yl - rl, -b * yh - rh) * ia) - pad
            qh = min(max(math.floor(f(f(xmax + cx - f(0.5)) / f(CS))) - cx0, -1), 4)
            ql = min(max(math.ceil(f(f(f(xmin + cx + f(0.5)) / f(CS)) - f(1))) - cx0, 0), 5)
            keep = ((1 << (qh + 1)) - 1) & ~((1 << ql) - 1)
        excl |= (allb & ~keep) << (4 * r)
    return excl


def bins_from_cells(cexcl, x0, y0, x1, y1):
    cx0, cy0, cx1, cy1 = x0 >> 3, y0 >> 3, x1 >> 3, y1 >> 3
    ncol, nrow = cx1 - cx0 + 1, cy1 - cy0 + 1
    sx, sy = min(4 - (cx0 & 3), ncol), min(4 - (cy0 & 3), nrow)
    col0 = (1 << sx) - 1; col1 = ((1 << ncol) - 1) & ~col0
    row0 = sum(0xF << (4 * r) for r in range(min(sy, nrow)))
    row1 = sum(0xF << (4 * r) for r in range(sy, nrow))
    inc = ~cexcl & 0xFFFF
    colm = lambda c: c | c << 4 | c << 8 | c << 12
    b = 0
    if inc & row0 & colm(col0) == 0: b |= 1
    if col1 and inc & row0 & colm(col1) == 0: b |= 2
    if row1 and inc & row1 & colm(col0) == 0: b |= 16
    if col1 and row1 and inc & row1 & colm(col1) == 0: b |= 32
    allb = (3 if col1 else 1) * (17 if row1 else 1)
    return b & ~1 if b == allb else b


def keep_one_bin(b, x0, y0, x1, y1):
    cols, rows = (x1 >> 5) - (x0 >> 5) + 1, (y1 >> 5) - (y0 >> 5) + 1
    if cols > 4 or rows > 4:
        return b
    allb = sum(((1 << cols) - 1) << (4 * r) for r in range(rows))
    return b & ~1 if b == allb else b


def covered(ax, ay, bx, by, cx, cy, X0, X1, Y0, Y1):
    """Any pixel centre of [X0, X1] x [Y0, Y1] inside q <= QMAX (float64)."""
    X, Y = np.meshgrid(np.arange(X0, X1 + 1) + 0.5 - float(cx), float(cy) - (np.arange(Y0, Y1 + 1) + 0.5))
    u = X * float(ax) + Y * float(ay); v = X * float(bx) + Y * float(by)
    return bool(((u * u + v * v) <= float(QMAX)).any())


def test_masks_conservative_and_keep_a_bin():
    rng = np.random.default_rng(7)
    checked = 0
    for _ in range(3000):
        r1 = f(rng.uniform(0.3, 70)); r2 = f(rng.uniform(0.05, 1) * r1); th = rng.uniform(0, np.pi)
        e1 = np.array([np.cos(th), np.sin(th)], np.float32); e2 = np.array([-e1[1], e1[0]], np.float32)
        ax, ay = e1 * f(3) / r1; bx, by = e2 * f(3) / r2
        cx, cy = f(rng.uniform(0, 1920)), f(rng.uniform(0, 1080))
        hx = r1 * abs(e1[0]) + r2 * abs(e2[0]) + 1; hy = r1 * abs(e1[1]) + r2 * abs(e2[1]) + 1
        x0, x1 = int(max(0, math.ceil(cx - hx - 0.5))), int(math.floor(cx + hx - 0.5))
        y0, y1 = int(max(0, math.ceil(cy - hy - 0.5))), int(math.floor(cy + hy - 0.5))
        if x1 < x0 or y1 < y0:
            continue
        e = ellipse_x(ax, ay, bx, by)
        small = (x1 >> 3) - (x0 >> 3) < 4 and (y1 >> 3) - (y0 >> 3) < 4
        m = cell_mask(e, cx, cy, x0, y0, x1, y1, 3 if small else 5)
        cexcl = m if small else 0
        bexcl = bins_from_cells(m, x0, y0, x1, y1) if small else keep_one_bin(m, x0, y0, x1, y1)
        for shift, ex in ((3, cexcl), (5, bexcl)):
            c0, r0 = x0 >> shift, y0 >> shift
            for bit in range(16):
                if not (ex >> bit) & 1:
                    continue
                q, r = bit & 3, bit >> 2
                X0 = max((c0 + q) << shift, x0); X1 = min(((c0 + q + 1) << shift) - 1, x1)
                Y0 = max((r0 + r) << shift, y0); Y1 = min(((r0 + r + 1) << shift) - 1, y1)
                assert X0 <= X1 and Y0 <= Y1, (shift, bit, x0, y0, x1, y1)  # bits only inside the rect
                assert not covered(ax, ay, bx, by, cx, cy, X0, X1, Y0, Y1), (shift, bit, x0, y0, x1, y1)
                checked += 1
        # a non-empty rect keeps at least one of its bins
        bx0, by0, bx1, by1 = x0 >> 5, y0 >> 5, x1 >> 5, y1 >> 5
        if bx1 - bx0 < 4 and by1 - by0 < 4:
            allb = sum(((1 << (bx1 - bx0 + 1)) - 1) << (4 * r) for r in range(by1 - by0 + 1))
            assert bexcl & allb != allb
    assert checked > 1000
