"""MLAB k-buffer mode (gaussian_splat.metal:201-361).

The C oracle (oracle/gs_oracle.c mlab_*) is pinned two ways: hand-derived
known answers, and an independent numpy restatement below that uses IEEE
float16 arithmetic (np.float16 ops are correctly rounded: products of two
halves are exact in float32, sums cannot create a double-rounding tie).
Parity with Metal itself is unpinned (no Metal runtime): the reference may
contract `back.rgb + front.rgb * back.a` into an fma."""
import numpy as np
import pytest

from oracle import oracle_py as O

H = np.float16


def mlab_numpy(frags):
    """Restatement of fragment_main + resolve_main with numpy float16."""
    L = [[H(0), H(0), H(0), H(1)] for _ in range(6)]
    D = [H(0)] * 6
    D[3] = H(1)  # depths01 cleared to (0,0,0,1) (instanced_splat_renderer.mm:540)
    for depth, r, g, b, a in frags:
        ha = H(a)
        nl = [H(r) * ha, H(g) * ha, H(b) * ha, H(1) - ha]
        nd = H(depth)
        for i in range(6):
            if nd >= D[i]:
                L[i], nl = nl, L[i]
                D[i], nd = nd, D[i]
        closer = nd >= D[5]
        front, back = (nl, L[5]) if closer else (L[5], nl)
        L[5] = [back[0] + front[0] * back[3], back[1] + front[1] * back[3], back[2] + front[2] * back[3],
                front[3] * back[3]]
        D[5] = nd if closer else D[5]
    C = [H(0), H(0), H(0)]
    at = H(1)
    for i in range(6):
        C = [C[c] + L[i][c] * at for c in range(3)]
        at = at * L[i][3]
    return np.array([C[0], C[1], C[2], H(1) - at], np.float32)


def test_mlab_known_answers():
    # one fragment: (rgb * a, a), half-rounded
    np.testing.assert_array_equal(O.composite_list([[2.0, 1.0, 0.5, 0.25, 0.5]], mode="mlab"),
                                  np.float32([0.5, 0.25, 0.125, 0.5]))
    # three fragments, depths 2, 5, 3: stored far-first (5, 3, 2), resolved
    # layer 0 first -> the same answer as the tile contract's S1 order
    np.testing.assert_array_equal(
        O.composite_list([[2.0, 1, 0, 0, 0.5], [5.0, 0, 1, 0, 0.5], [3.0, 0, 0, 1, 0.5]], mode="mlab"),
        np.float32([0.125, 0.5, 0.25, 0.875]))
    # empty pixel
    np.testing.assert_array_equal(O.composite_list(np.zeros((0, 5)), mode="mlab"), np.zeros(4, np.float32))
    # the depth-1 sentinel of the cleared k-buffer: fragments nearer than 1
    # never pass slot 3, so the 5th such fragment merges into slot 5 (under)
    fr = [[0.5, 1, 0, 0, 0.5]] * 5
    got = O.composite_list(fr, mode="mlab")
    np.testing.assert_array_equal(got, mlab_numpy(fr))
    assert got[3] > 0.9  # all five contribute


@pytest.mark.parametrize("seed", range(6))
def test_mlab_oracle_matches_numpy_float16(seed):
    rng = np.random.default_rng(seed)
    for _ in range(200):
        n = int(rng.integers(0, 16))
        depth = rng.choice([0.3, 0.9, 1.0, 1.5, 2.0, 4.0, 7.5], size=n) if rng.random() < 0.5 else \
            rng.uniform(0.1, 9.0, size=n)
        frags = np.column_stack([depth, rng.random(n), rng.random(n), rng.random(n),
                                 rng.uniform(0.001, 0.99, n)]).astype(np.float32)
        got = O.composite_list(frags, mode="mlab")
        np.testing.assert_array_equal(got.view(np.uint32), mlab_numpy(frags).view(np.uint32))
