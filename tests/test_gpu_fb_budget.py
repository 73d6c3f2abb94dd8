"""Fixed-base tables built on first use (csrc/commit.hip fb_default_c): the widest window <= 16
bits that fits what is left of the context's budget for such tables (VKZG_FB_BUDGET_GB, default
20 GB) -- 16 bits (17.2 GB) for the first 257-point table of a context, narrower ones after it --
and the same commitments whatever window a table got."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_auto_windows_follow_the_context_budget():
    import vkzg
    e = vkzg.Engine("bn254")
    try:
        n = 257
        tabs = [e.random_bases(n, seed=7) for _ in range(3)]  # the same bases three times
        sc = vkzg.random_scalars("bn254", 2 * n, np.random.default_rng(5))  # 2 commits of width 257
        outs, geos = [], []
        for t in tabs:
            assert e.fixed_base_geometry(t)[0] == 0  # none yet: built by the first commit
            out, inf = e.msm_batch(t, sc, n)
            outs.append((out.copy(), inf.copy()))
            geos.append(e.fixed_base_geometry(t))
        assert geos[0][:2] == (16, 16), geos
        assert geos[1][0] < 16 and geos[2][0] <= geos[1][0], geos
        assert sum(e.fixed_base_table_bytes(t) for t in tabs) <= 20e9 + 2 * 0.2e9
        for out, inf in outs[1:]:
            assert np.array_equal(out, outs[0][0]) and np.array_equal(inf, outs[0][1])
    finally:
        e.close()


def test_auto_budget_returns_when_a_table_is_precomputed_explicitly():
    """a first-use table that is later precomputed explicitly (vc_fixed_base_precompute) stops
    counting against the budget: the next first-use table gets 16-bit windows again"""
    import vkzg
    e = vkzg.Engine("bn254")
    try:
        n = 257
        sc = vkzg.random_scalars("bn254", n, np.random.default_rng(9))
        a = e.random_bases(n, seed=3)
        want = e.msm_batch(a, sc, n)
        assert e.fixed_base_geometry(a)[0] == 16
        e.fixed_base_precompute(a, 8)               # explicit: 134 MB, outside the budget
        assert e.fixed_base_geometry(a)[0] == 8
        b = e.random_bases(n, seed=3)
        got = e.msm_batch(b, sc, n)
        assert e.fixed_base_geometry(b)[0] == 16
        assert np.array_equal(got[0], want[0]) and np.array_equal(e.msm_batch(a, sc, n)[0], want[0])
    finally:
        e.close()
