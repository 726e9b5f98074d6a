"""tools/replay_potrf.py: the rank-replay harness compiles and runs every rank's distributed
Cholesky program in ONE process (transport replaced by a timing model) -- here on CPU with the
no-op model, checking that each rank's program runs to the end and issues the batches that the
real transport would."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tool():
    spec = importlib.util.spec_from_file_location("replay_potrf", os.path.join(ROOT, "tools", "replay_potrf.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize("grid,uplo", [((2, 4), 122), ((2, 1), 122), ((1, 2), 121), ((2, 2), 121)])
def test_replay_every_rank_cpu(grid, uplo, monkeypatch):
    monkeypatch.setenv("DPLASMA_POTRF_DEFER_MIN_TILES", "3")
    m = _tool()
    import dplasma_amd as dp
    from dplasma_amd.parallel import comm
    base = dp.Context(device="cpu")
    be = m.ReplayBackend("cpu", 50.0, 15.0, 4)
    comm.set_backend(be)
    try:
        P, Q = grid
        for r in range(P * Q):
            t, enq = m.replay_rank(base, P, Q, r, 19 * 12, 19, uplo, 1, be)
            assert t >= 0
        assert be.stats["batches"] > 0
    finally:
        comm.set_backend(None)


def _hqr_tool():
    spec = importlib.util.spec_from_file_location("replay_hqr", os.path.join(ROOT, "tools", "replay_hqr.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize("grid,a", [((2, 4), 0), ((2, 2), 2), ((4, 1), 0)])
def test_replay_hqr_every_rank_cpu(grid, a):
    """tools/replay_hqr.py (BASELINE config 4 model): every rank's stacked-domain HQR program runs to the
    end with its exchanges (V/T broadcasts, TT partner transfers, partial-W sums) modelled."""
    m, mp = _hqr_tool(), _tool()
    import dplasma_amd as dp
    from dplasma_amd.parallel import comm
    base = dp.Context(device="cpu")
    be = mp.ReplayBackend("cpu", 50.0, 15.0, 4)
    comm.set_backend(be)
    try:
        P, Q = grid
        for r in range(P * Q):
            t, enq = m.replay_rank(base, P, Q, r, 10 * 16, 16, 8, (1, 1, a, -1, 0), 0, mp.fake_rank_context)
            assert t >= 0
        assert be.stats.get("sync_bcast", 0) + be.stats.get("sync_p2p", 0) > 0
    finally:
        comm.set_backend(None)
