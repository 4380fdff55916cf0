"""GPU tests of the library's own RCCL communicator (dh_comm_*, dh_allgather_best: SURVEY 8(b),
8(e)).  One GPU per box here, and RCCL refuses two ranks on one device, so these run a world of
one: a real communicator init, broadcast and all-gather through RCCL, and the whole
calibrate_sharded path (records encoded, gathered, decoded, best start chosen) over it.  The
multi-rank logic above the transport is the torch.distributed path's, tested with gloo ranks in
tests/test_distributed.py."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    from dhcos import _native
    if _native.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X box")
    c = _native.Comm(_native.default_context(), _native.comm_id(), 1, 0)
    yield c
    c.close()


def test_comm_broadcast_and_allgather_keep_bits(comm):
    from dhcos import _native
    rs = np.random.RandomState(3)
    buf = rs.normal(size=37)
    buf[5] = np.nan
    out = comm.broadcast(buf.copy(), 0)
    assert np.array_equal(out.view(np.int64), buf.view(np.int64))
    rec = rs.normal(size=(6, 9))
    rec[:, 1] = [4, 0, -1, 2, 1, 3]                   # start indices, one padding row
    rec[:, 2] = [0.3, np.nan, 0.1, 0.3, 0.2, np.inf]
    allr, best = comm.allgather_best(rec, 1, 2)
    assert np.array_equal(allr.view(np.int64), rec.view(np.int64))
    assert best == _native.best_start(rec, 1, 2) == 1        # start 0 is NaN; 1 (0.2) beats 2, 4


def test_calibrate_sharded_over_native_comm_equals_calibrate(comm, calib_golden):
    """calibrate_sharded through dh_comm_broadcast / dh_allgather_best (no torch.distributed):
    the result, n_calls / best_loss and the np.random continuation of calibrate()."""
    import dhcos
    from dhcos import distributed as D
    market = calib_golden["test_market"]
    np.random.seed(0)
    want = dhcos.DoubleHestonJumpCalibrator(100.0, 0.05, market)
    w = want.calibrate(300, 3)
    after = np.random.rand()
    np.random.seed(0)
    cal = dhcos.DoubleHestonJumpCalibrator(100.0, 0.05, market)
    got = D.calibrate_sharded(cal, 300, 3, comm=comm)
    assert np.random.rand() == after
    assert got.final_loss == w.final_loss and got.iterations == w.iterations
    assert got.message == w.message and got.parameters == w.parameters
    np.testing.assert_array_equal(got.model_prices, w.model_prices)
    assert (cal.n_calls, cal.best_loss) == (want.n_calls, want.best_loss)


def test_generate_sharded_over_native_comm_equals_generator(comm, tmp_path):
    """generate_sharded through dh_comm_broadcast / dh_comm_allgather: the generator's output and
    its np.random continuation."""
    from dhcos import distributed as D
    from dhcos import generator as G
    np.random.seed(5)
    want = G.generate_synthetic_calibrations(48, str(tmp_path / "a.pkl"), N=64, as_arrays=True,
                                             verbose=False)
    after = np.random.rand()
    np.random.seed(5)
    got = D.generate_sharded(48, str(tmp_path / "b.pkl"), N=64, as_arrays=True, verbose=False,
                             comm=comm)
    assert np.random.rand() == after
    assert set(got) == set(want)
    for k in want:
        a, b = np.asarray(want[k]), np.asarray(got[k])
        assert a.shape == b.shape and (a == b).all() or np.array_equal(a, b, equal_nan=True), k
