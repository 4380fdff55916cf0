"""The fused request kernel's loss hand-offs and table maps give the same bits.

A fused loss request sums each param set's tile partials in one of three ways ($DHCOS_DEFER: 2, the
default, the grid's last blocks from epoch-tagged granules; 1, a summing launch after the grid;
0, the ticket hand-off in every block), and one-round grids map blocks to tables by XCD
($DHCOS_XCD_REMAP=1, the default; =2 multi-round grids too).  Every form reads the same partials in the same order and butterfly, and the map
is a bijection, so sse and n_bad must be bit for bit the same -- on a multi-round grid (C3's shape:
4,200 tables) and a one-round grid (C2's: 448), with an invalid price in the market (n_bad > 0),
and over back-to-back requests (the granules' epochs).  Each setting gets a context of its own (the
switches are read once per context).  Reference: lbfgs_calibrator.py:128-164."""
import os

import numpy as np
import pytest

from test_gpu_fullsize import GEN_HI, GEN_LO

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    from dhcos import _native
    if _native.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X box")
    return _native


def grid(nK, nT, S0=100.0, r=0.03, seed=5):
    kk, tt = np.meshgrid(np.linspace(0.8, 1.2, nK) * S0, np.linspace(0.1, 2.0, nT))
    K, T = kk.ravel(), tt.ravel()
    call = K >= S0
    rs = np.random.RandomState(seed)
    mkt = 10.0 * rs.uniform(0.5, 1.5, K.size)
    mkt[7] = -1.0                                  # a market price the loss divides by
    recs = np.zeros((42, 16))
    recs[:, :13] = GEN_LO + (GEN_HI - GEN_LO) * rs.rand(42, 13)
    recs[:, 13], recs[:, 14] = S0, r
    recs[5, 0] = np.nan                            # a NaN parameter: NaN prices, n_bad > 0
    return K, T, call, mkt, recs


def losses(native, env, K, T, call, mkt, recs, N, reps=3):
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        ctx = native.Context(0)
        surf = native.Surface(ctx, K, T, call, mkt)
        out = [surf.loss_terms(recs, N)[:2] for _ in range(reps)]
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    for sse, bad in out[1:]:                       # back-to-back requests: the same bits
        assert np.array_equal(sse.view(np.int64), out[0][0].view(np.int64))
        assert np.array_equal(bad, out[0][1])
    return out[0]


@pytest.mark.parametrize("nK, nT, N", [(100, 100, 512), (32, 32, 256)])
def test_loss_modes_and_maps_bitwise(native, nK, nT, N):
    K, T, call, mkt, recs = grid(nK, nT)
    want_sse, want_bad = losses(native, {"DHCOS_DEFER": "0", "DHCOS_XCD_REMAP": "0"},
                                K, T, call, mkt, recs, N)
    assert (want_bad[5] > 0) and (want_bad > 0).sum() >= 1
    for env in ({"DHCOS_DEFER": "1", "DHCOS_XCD_REMAP": "0"},
                {"DHCOS_DEFER": "2", "DHCOS_XCD_REMAP": "0"},
                {"DHCOS_DEFER": "2", "DHCOS_XCD_REMAP": "1"},
                {"DHCOS_DEFER": "2", "DHCOS_XCD_REMAP": "2"}):    # by XCD on multi-round grids too
        sse, bad = losses(native, env, K, T, call, mkt, recs, N)
        assert np.array_equal(bad, want_bad), env
        assert np.array_equal(sse.view(np.int64), want_sse.view(np.int64)), \
            (env, np.flatnonzero(sse.view(np.int64) != want_sse.view(np.int64))[:5])
