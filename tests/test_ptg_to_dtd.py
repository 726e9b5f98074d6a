"""PTG -> DTD re-execution (the reference's ``--mca mca_pins ptg_to_dtd`` test mode): with
DPLASMA_PTG_TO_DTD=1 every tile DAG is re-inserted task by task through the DTD front end, which
rediscovers the dependencies from the access modes -- results must be identical."""
import pytest
import torch

import dplasma_amd as dp
from dplasma_amd.models import qr_panel
from dplasma_amd.runtime import dag as dagmod
from helpers import rel_err, run_distributed


@pytest.fixture(scope="module")
def ctx():
    return dp.init(device="cpu")


@pytest.fixture
def ptg_flag():
    old = dagmod.PTG_TO_DTD[0]

    def set_(v):
        dagmod.PTG_TO_DTD[0] = v
    yield set_
    dagmod.PTG_TO_DTD[0] = old


def _qr(ctx, tree=False):
    A = dp.block_cyclic(ctx, torch.float64, 24, 24, 130, 100)
    dp.plrnt(ctx, A, 5)
    TS = dp.block_cyclic(ctx, torch.float64, 8, 24, A.mt * 8, A.nt * 24, name="TS")
    TT = dp.block_cyclic(ctx, torch.float64, 8, 24, A.mt * 8, A.nt * 24, name="TT")
    with qr_panel.engine("tile"):
        if tree:
            t = dp.hqr_init(dp.dplasmaNoTrans, A, 1, 0, 2, 1)
            tp = dp.geqrf_param_New(ctx, t, A, TS, TT)
        else:
            tp = dp.geqrf_New(ctx, A, TS)
        tp.execute(ctx)
    return tp, A.to_dense_local(), TS.to_dense_local()


@pytest.mark.parametrize("tree", [False, True])
def test_qr_through_dtd(ctx, tree, ptg_flag):
    ptg_flag(False)
    tp0, a0, t0 = _qr(ctx, tree)
    ptg_flag(True)
    tp1, a1, t1 = _qr(ctx, tree)
    assert getattr(tp1, "ptg_to_dtd", False) and not getattr(tp0, "ptg_to_dtd", False)
    assert rel_err(a1, a0) < 1e-14 and rel_err(t1, t0) < 1e-14


def test_incpiv_lu_through_dtd(ctx, ptg_flag):
    out = []
    for flag in (False, True):
        ptg_flag(flag)
        A = dp.block_cyclic(ctx, torch.float64, 32, 32, 140, 140)
        dp.plrnt(ctx, A, 7)
        L = dp.incpiv_L_descriptor(ctx, A, 8)
        IP = dp.incpiv_ipiv_descriptor(ctx, A)
        tp = dp.getrf_incpiv_New(ctx, A, L, IP)
        assert getattr(tp, "ptg_to_dtd", False) == flag
        assert tp.execute(ctx) == 0
        out.append((A.to_dense_local(), IP.to_dense_local()))
    assert rel_err(out[0][0], out[1][0]) < 1e-14 and torch.equal(out[0][1], out[1][1])


def _worker(rank, world, P):
    import dplasma_amd as dp
    from dplasma_amd.runtime import dag as dagmod
    ctx = dp.init(device="cpu", P=P)
    dagmod.PTG_TO_DTD[0] = True
    _, a, _ = _qr(ctx)
    return a


def test_qr_through_dtd_distributed():
    out = run_distributed(_worker, 2, 2)
    ctx = dp.init(device="cpu")
    _, a0, _ = _qr(ctx)
    assert rel_err(out[0] + out[1], a0) < 1e-12


@pytest.mark.gpu
def test_gpu_incpiv_lu_through_dtd(ptg_flag):
    g = dp.init(device="cuda:0")
    out = []
    for flag in (False, True):
        ptg_flag(flag)
        A = dp.block_cyclic(g, torch.float64, 128, 128, 700, 700)
        dp.plrnt(g, A, 7)
        L = dp.incpiv_L_descriptor(g, A, 32)
        IP = dp.incpiv_ipiv_descriptor(g, A)
        tp = dp.getrf_incpiv_New(g, A, L, IP)
        assert getattr(tp, "ptg_to_dtd", False) == flag
        assert tp.execute(g) == 0
        out.append((A.to_dense_local().cpu(), IP.to_dense_local().cpu()))
    assert rel_err(out[0][0], out[1][0]) < 1e-13 and torch.equal(out[0][1], out[1][1])
