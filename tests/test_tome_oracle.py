"""CPU: pin the ToMe oracle (canonical C + literal numpy) against the hand-derived KATs of
SURVEY.md §8c (derived from token_compression.py:54-129; the reference has no ToMe test of its
own) and against each other."""
import numpy as np
import pytest

from oracle import tome as O


def _rows(x, idx):
    return np.stack([x[i] for i in idx])


def test_kat1_ties_literal_and_canon():
    metric = np.ones((1, 8, 4), np.float32)
    x = np.random.default_rng(0).standard_normal((1, 8, 5)).astype(np.float32)
    # literal
    merge, unm, src, dst = O.literal_bipartite_soft_matching(metric, 2)
    assert unm.tolist() == [[1, 0]] and src.tolist() == [[3, 2]] and dst.tolist() == [[0, 0]]
    out, size = O.literal_merge_wavg(merge, x)
    exp = np.stack([x[0, 2], x[0, 0], (x[0, 1] + x[0, 6] + x[0, 4]) / 3, x[0, 3], x[0, 5], x[0, 7]])
    np.testing.assert_allclose(out[0], exp, rtol=1e-6)
    assert size[0, :, 0].tolist() == [1, 1, 3, 1, 1, 1]
    # canonical C
    cu, cs, cd, _ = O.canon_match(metric, 2)
    assert (cu == unm).all() and (cs == src).all() and (cd == dst).all()
    co, csz = O.canon_merge_wavg(x, None, cu, cs, cd, 2)
    np.testing.assert_allclose(co, out, rtol=1e-6)
    assert csz[0].tolist() == [1, 1, 3, 1, 1, 1]


def test_kat1_r_clamped():
    metric = np.ones((1, 8, 4), np.float32)
    x = np.random.default_rng(1).standard_normal((1, 8, 3)).astype(np.float32)
    merge, unm, src, dst = O.literal_bipartite_soft_matching(metric, 10)  # clamps to 4
    out, size = O.literal_merge_wavg(merge, x)
    exp = np.stack([(x[0, 1] + x[0, 6] + x[0, 4] + x[0, 2] + x[0, 0]) / 5, x[0, 3], x[0, 5], x[0, 7]])
    np.testing.assert_allclose(out[0], exp, rtol=1e-6)
    assert size[0, :, 0].tolist() == [5, 1, 1, 1]
    cu, cs, cd, _ = O.canon_match(metric, 4)
    assert (cs == src).all() and (cd == dst).all() and cu.shape == (1, 0)


@pytest.mark.parametrize("r,rows,sizes", [
    (1, ["x2", "x4", "(x1+x0)/2", "x3", "x5"], [1, 1, 2, 1, 1]),
    (2, ["x4", "(x1+x0)/2", "(x3+x2)/2", "x5"], [1, 2, 2, 1]),
])
def test_kat2_distinct(r, rows, sizes):
    metric = np.array([[[1, 0], [1, .1], [0, 1], [.2, 1], [1, 1], [-1, 0]]], np.float32)
    x = np.random.default_rng(2).standard_normal((1, 6, 4)).astype(np.float32)
    merge, unm, src, dst = O.literal_bipartite_soft_matching(metric, r)
    out, size = O.literal_merge_wavg(merge, x)
    env = {f"x{i}": x[0, i] for i in range(6)}
    exp = np.stack([eval(e, {}, env) for e in rows])
    np.testing.assert_allclose(out[0], exp, rtol=1e-6)
    assert size[0, :, 0].tolist() == sizes
    _, _, _, nmax = O.canon_match(metric, r)
    np.testing.assert_allclose(nmax[0], [.99504, .98058, .83205], atol=1e-5)
    cu, cs, cd, _ = O.canon_match(metric, r)
    co, csz = O.canon_merge_wavg(x, None, cu, cs, cd, r)
    np.testing.assert_allclose(co, out, rtol=1e-6)
    assert csz[0].tolist() == sizes


def test_r_zero_is_do_nothing():
    assert O.literal_bipartite_soft_matching(np.ones((1, 2, 3), np.float32), 0) is None
    assert O.literal_bipartite_soft_matching(np.ones((1, 3, 3), np.float32), 5, True, True) is None


@pytest.mark.parametrize("t,c,r,flags", [(256, 64, 16, 0), (257, 64, 16, 0), (64, 32, 8, 1),
                                          (64, 32, 8, 2), (64, 32, 8, 3), (31, 6, 7, 0)])
def test_canon_matches_literal_random(t, c, r, flags):
    rng = np.random.default_rng(t * 7 + c + flags)
    n = 3
    metric = rng.standard_normal((n, t, c)).astype(np.float32)
    x = rng.standard_normal((n, t, 16)).astype(np.float32)
    size = rng.integers(1, 5, (n, t)).astype(np.float32)
    lit = O.literal_bipartite_soft_matching(metric, r, bool(flags & 1), bool(flags & 2))
    merge, unm, src, dst = lit
    cu, cs, cd, _ = O.canon_match(metric, r, flags)
    # random gaussian data: no near-ties, so ulp differences cannot reorder
    assert (cu == unm).all() and (cs == src).all() and (cd == dst).all()
    lo, ls = O.literal_merge_wavg(merge, x, size[..., None])
    co, csz = O.canon_merge_wavg(x, size, cu, cs, cd, r, flags)
    np.testing.assert_allclose(co, lo, rtol=2e-6, atol=1e-6)
    np.testing.assert_array_equal(csz, ls[..., 0])


def test_plain_sum_and_no_scatter_modes():
    rng = np.random.default_rng(5)
    metric = rng.standard_normal((2, 20, 8)).astype(np.float32)
    x = rng.standard_normal((2, 20, 4)).astype(np.float32)
    merge, unm, src, dst = O.literal_bipartite_soft_matching(metric, 5)
    cu, cs, cd, _ = O.canon_match(metric, 5)
    co, _ = O.canon_merge_wavg(x, None, cu, cs, cd, 5, flags=4)
    np.testing.assert_allclose(co, merge(x, "sum"), rtol=1e-6)
    co, _ = O.canon_merge_wavg(x, None, cu, cs, cd, 5, flags=4 | 8)
    np.testing.assert_allclose(co, merge(x, "none"), rtol=1e-6)


def test_heads_metric_is_sum_over_heads():
    rng = np.random.default_rng(9)
    k = rng.standard_normal((2, 40, 6, 16)).astype(np.float32)
    a = O.canon_match(k, 6)
    b = O.canon_match(k.sum(axis=2, dtype=np.float64).astype(np.float32), 6)
    # different summation precision, same generic-data matching
    for u, v in zip(a[:3], b[:3]):
        assert (u == v).all()


def test_pos_map_and_bwd_are_jacobian_transpose():
    rng = np.random.default_rng(11)
    n, t, D, r = 2, 30, 3, 6
    metric = rng.standard_normal((n, t, 5)).astype(np.float32)
    size = rng.integers(1, 4, (n, t)).astype(np.float32)
    cu, cs, cd, _ = O.canon_match(metric, r)
    pos = O.canon_pos_map(cu, cs, cd, t, r)
    assert (pos >= 0).all()
    _, so = O.canon_merge_wavg(np.zeros((n, t, D), np.float32), size, cu, cs, cd, r)
    g = rng.standard_normal((n, t - r, D)).astype(np.float32)
    gi = O.canon_merge_bwd(g, size, so, pos)
    # numerical Jacobian-vector check: <g, merge(x + e)> - <g, merge(x)> = <gi, e> (linear map)
    x = rng.standard_normal((n, t, D)).astype(np.float64)
    e = rng.standard_normal((n, t, D)).astype(np.float64)
    f = lambda z: O.canon_merge_wavg(z.astype(np.float32), size, cu, cs, cd, r)[0].astype(np.float64)
    lhs = (g * (f(x + e) - f(x))).sum()
    rhs = (gi * e).sum()
    assert abs(lhs - rhs) < 1e-4 * max(1.0, abs(rhs))
