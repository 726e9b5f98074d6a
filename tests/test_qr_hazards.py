"""Cross-stream buffer hazards of the distributed stacked-domain QR (models/qr_panel.py, P x Q, look-ahead): the same
instrumented run as tests/test_lu_hazards.py on the HQR task graph -- qr_panel / qr_next on the GPU's "panel" stream,
qr_rest on "update" -- every pair of tasks on different streams touching one scratch buffer (panel / V / T buffers,
W partial sums and their exchange buffers), one writing, must be ordered by the graph."""
import torch

from helpers import run_distributed
from test_lu_hazards import _hazards, instrumented_run

QR_STREAMS = (("qr_panel(", "panel"), ("qr_next(", "panel"), ("qr_rest(", "update"), ("qr_vsend(", "vsend"))


def _worker(rank, world, N, NB, a, share=False):
    import dplasma_amd as dp
    from dplasma_amd.models import qrtree
    ctx = dp.init(device="cpu", P=2)
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plrnt(ctx, A, 3872)
    ib = 8
    TS = dp.block_cyclic(ctx, torch.float64, ib, NB, A.mt * ib, N)
    TT = dp.block_cyclic(ctx, torch.float64, ib, NB, A.mt * ib, N)
    tree = qrtree.hqr_init(dp.dplasmaNoTrans, A, qrtree.GREEDY_TREE, qrtree.GREEDY_TREE, a or -(-A.mt // 2), 2)
    tp = dp.geqrf_param_New(ctx, tree, A, TS, TT)
    st = tp._state
    if share:   # negative control: next and rest sum their W partials in the same work buffers
        st.wn = st.wr
    names = [t.name for t in tp.tasks]
    info, graph, acc = instrumented_run(ctx, tp, st, A)
    return info, graph, acc, bool(getattr(st, "la", False)), names[:3]


def test_hqr_2x4_cross_stream_buffer_hazards():
    for a in (0, 2):
        out = run_distributed(_worker, 8, 128, 16, a)
        found = []
        for r in range(8):
            info, graph, acc, la, names = out[r]
            assert la, names
            found += [(r,) + h for h in _hazards(graph, acc, QR_STREAMS)]
        assert not found, (a, found[:20])


def test_hqr_hazard_checker_negative_control():
    out = run_distributed(_worker, 8, 128, 16, 0, True)
    found = []
    for r in range(8):
        info, graph, acc, la, names = out[r]
        found += [(r,) + h for h in _hazards(graph, acc, QR_STREAMS)]
    assert any({h[2][:7], h[3][:7]} == {"qr_next", "qr_rest"} for h in found), found[:10]
