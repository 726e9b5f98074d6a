"""Rank-consistent use of the several RCCL communicators (urgent / bulk / row / col groups).

Each communicator runs its operations in issue order on its own stream, and RCCL point-to-point
operations between two ranks pair up in issue order on a communicator.  The distributed engines post
transfers from the same SPMD program on every rank (the taskpool issues its communicating tasks in
program order under every scheduler policy), so (1) on every communicator the messages a sends to b and
those b receives from a pair up in order, (2) every member issues the same collectives in the same order,
and (3) the batches of all communicators follow one global order of task labels -- no two ranks can wait
on each other's batches in a cycle.  These tests record every transfer of POTRF, SUMMA GEMM and HQR on a
2 x 4 world of gloo ranks (parallel.comm.record) and check the three conditions (parallel.comm.check_order);
the negative tests show that a permuted order is caught."""
import copy

import pytest
import torch

from dplasma_amd.parallel import comm
from helpers import run_distributed

pytestmark = pytest.mark.slow


def _potrf_w(rank, world):
    import dplasma_amd as dp
    from dplasma_amd.parallel import comm as c
    ctx = dp.init(device="cpu", P=2)
    A = dp.block_cyclic(ctx, torch.float64, 16, 16, 160, 160)
    dp.plghe(ctx, 160.0, dp.dplasmaLower, A, 3872)
    c.record(True)
    info = dp.potrf(ctx, dp.dplasmaLower, A)
    return info, c.record(False)


def _gemm_w(rank, world):
    import dplasma_amd as dp
    from dplasma_amd.parallel import comm as c
    ctx = dp.init(device="cpu", P=2)
    ctx.info.set("DPLASMA:GEMM:look_ahead", "2")
    A = dp.block_cyclic(ctx, torch.float64, 16, 16, 96, 112)
    B = dp.block_cyclic(ctx, torch.float64, 16, 16, 112, 80)
    C = dp.block_cyclic(ctx, torch.float64, 16, 16, 96, 80)
    for X, s in ((A, 1), (B, 2), (C, 3)):
        dp.plrnt(ctx, X, s)
    c.record(True)
    dp.gemm(ctx, dp.dplasmaNoTrans, dp.dplasmaNoTrans, 0.5, A, B, -0.5, C)
    return 0, c.record(False)


def _hqr_w(rank, world):
    import dplasma_amd as dp
    from dplasma_amd.models import qr_panel
    from dplasma_amd.parallel import comm as c
    ctx = dp.init(device="cpu", P=2)
    dt = torch.float64
    A = dp.block_cyclic(ctx, dt, 8, 8, 68, 36)
    dp.plrnt(ctx, A, 3)
    TS = dp.block_cyclic(ctx, dt, 4, 8, A.mt * 4, A.nt * 8)
    TT = dp.block_cyclic(ctx, dt, 4, 8, A.mt * 4, A.nt * 8)
    tree = dp.hqr_init(dp.dplasmaNoTrans, A, dp.dplasma_GREEDY_TREE, dp.dplasma_BINARY_TREE, 2, 2)
    c.record(True)
    with qr_panel.engine("panel"):
        dp.geqrf_param(ctx, tree, A, TS, TT)
    return 0, c.record(False)


def _getrf_w(rank, world):
    """getrf_ptgpanel on 2 x 4 with the point-to-point interchanges (next column / rest / left on three
    communicators, look-ahead): the recorded order must satisfy the same three conditions."""
    import dplasma_amd as dp
    from dplasma_amd.parallel import comm as c
    ctx = dp.init(device="cpu", P=2)
    A = dp.block_cyclic(ctx, torch.float64, 16, 16, 128, 128)
    dp.plrnt(ctx, A, 3872)
    IP = dp.ptgpanel_ipiv_descriptor(ctx, A)
    c.record(True)
    info = dp.getrf_ptgpanel(ctx, A, IP)
    return info, c.record(False)


@pytest.fixture(scope="module")
def logs():
    out = {}
    for name, fn in (("potrf", _potrf_w), ("gemm", _gemm_w), ("hqr", _hqr_w), ("getrf", _getrf_w)):
        res = run_distributed(fn, 8)
        assert all(res[r][0] == 0 for r in range(8))
        out[name] = {r: res[r][1] for r in range(8)}
    return out


@pytest.mark.parametrize("alg", ["potrf", "gemm", "hqr", "getrf"])
def test_comm_order_consistent(logs, alg):
    log = logs[alg]
    assert sum(len(v) for v in log.values()) > 0
    comms = {g for v in log.values() for _, g, _, _ in v}
    if alg == "potrf":     # the dataflow transport really uses several communicators
        assert len(comms) >= 2, comms
    if alg == "getrf":
        # rows cross process rows point to point (next column urgent, rest / left on the bulk communicators);
        # no all-reduce of the staging buffer is left
        kinds = {(g, k) for v in log.values() for _, g, k, _ in v}
        assert ("urgent", "p2p") in kinds and ("bulk0", "p2p") in kinds and ("bulk1", "p2p") in kinds, kinds
        assert not any(k == "allreduce" and g.startswith("col") for g, k in kinds), kinds
    comm.check_order(log)


@pytest.mark.parametrize("alg", ["potrf", "gemm", "hqr", "getrf"])
def test_comm_order_detects_permutation(logs, alg):
    """Swapping two point-to-point batches of one rank (different tasks) must fail the check: either the
    messages no longer pair up in order on their communicator, or the swap creates a wait cycle."""
    log = logs[alg]
    for r in range(8):
        seq = log[r]
        idx = [i for i, (lab, g, kind, b) in enumerate(seq) if kind == "p2p" and b]
        for a in range(len(idx)):
            for b in range(a + 1, len(idx)):
                i, j = idx[a], idx[b]
                if seq[i][0] == seq[j][0]:
                    continue
                if seq[i][1] != seq[j][1] or seq[i][1:] == seq[j][1:]:
                    # batches on different communicators may legitimately go in either order; two identical batches
                    # on one communicator cannot be told apart by any transport
                    continue
                bad = copy.deepcopy(log)
                bad[r][i], bad[r][j] = bad[r][j], bad[r][i]
                with pytest.raises(AssertionError):
                    comm.check_order(bad)
                return
    pytest.skip("no two batches with different labels on one rank")
