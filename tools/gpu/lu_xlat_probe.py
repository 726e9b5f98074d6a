"""Per-column cost of the distributed LU panel's cross-rank pivot hand-off, MEASURED (replaces the assumed --xlat 6 us
of tools/replay_lu.py; VERDICT r5 Next #1 / Weak #8).

Two ranks of one process column are emulated inside ONE process on ONE MI355X: rank q runs the distributed panel
kernel (csrc/kernels/lu_dist.hip, the production code path ops.lu_dist_ops.DistPanelLU) on its own rows of a real
N x 512 panel (tile rows m with m % 2 == q, plus the replicated diagonal tile) on a stream confined to half of the
CUs, and the two exchange every column's candidate through uncached exchange slots exactly as two GPUs do over xGMI
(system-scope stores + epoch flags); the pivots must equal LAPACK's (torch.linalg.lu_factor) on the whole panel.
Three timings per panel size:
  two     -- both ranks concurrently, each on 128 CUs, exchanging (the emulated grid)
  one     -- rank 0 alone on the same 128 CUs, exchanging with itself (what each rank pays without a peer)
  full    -- rank 0 alone on the whole GPU, exchanging with itself (what tools/replay_lu.py runs per rank)
xlat = (two - one) / columns is the cost of a real peer: the skew between the ranks plus the hand-off through memory
outside the rank's CUs; the replay adds it (plus an explicit xGMI latency increment, --xgmi) to every column.

  python tools/gpu/lu_xlat_probe.py [N] [k ...]"""
import ctypes
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

import dplasma_amd as dp  # noqa: E402
from dplasma_amd.ops import _lib, lu_dist_ops  # noqa: E402


class _Xc:
    def __init__(self, me, P, bases, slot_bytes, dev):
        self.group, self.me, self.P, self.slot_bytes = None, me, P, slot_bytes
        self.epoch = 1
        self.ok = True
        self.peers = torch.tensor(bases, dtype=torch.int64, device=dev)


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    ks = [int(x) for x in sys.argv[2:]] or [2, 64, 112]
    NB = 512
    ctx = dp.init(device="cuda:0")
    dev = ctx.device
    lib = _lib.load()
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    half = ncu // 2
    sA = ctx.streams[ctx.masked_stream("xlatA", range(0, half))]
    sB = ctx.streams[ctx.masked_stream("xlatB", range(half, ncu))]
    sF = ctx.streams["update"]
    slot = int(lib.dpl_lu_dist_slot_bytes(_lib.prec_code(torch.float64), NB))
    bases = []
    for _ in range(3):
        p, h = ctypes.c_void_p(), (ctypes.c_char * int(lib.dpl_ipc_handle_bytes()))()
        _lib.check(lib.dpl_xchg_alloc(2 * 2 * slot, ctypes.byref(p), h), "xchg_alloc")
        bases.append(p.value)
    nt = N // NB
    print(f"N={N} NB={NB}: two emulated ranks on CUs [0,{half}) / [{half},{ncu}), one process", flush=True)
    for k in ks:
        r0 = k * NB
        mp = N - r0
        g = torch.Generator(device=dev).manual_seed(3872 + k)
        pan = torch.randn(NB, mp, dtype=torch.float64, device=dev, generator=g).t()   # mp x NB, column-major
        ref_piv = torch.linalg.lu_factor(pan.cpu())[1].numpy() - 1                      # LAPACK pivots, 0-based
        ranks = []
        for q in range(2):
            own = [m for m in range(k + 1, nt) if m % 2 == q]
            rows = list(range(0, NB)) + [(m - k) * NB + i for m in own for i in range(NB)]
            ld = len(rows)
            idx = torch.tensor(rows, device=dev)
            buf0 = pan.index_select(0, idx).t().contiguous().view(-1)         # column-major, ld rows
            lrel = [(m - k) * NB + i for m in own for i in range(NB)]
            pv = buf0.clone()
            plu = lu_dist_ops.DistPanelLU(pv, ld, ld, NB, NB, q == k % 2, lrel)
            ranks.append(dict(buf0=buf0, pv=pv, plu=plu, ws=lu_dist_ops.dist_workspace(NB, dev),
                              cnt=torch.zeros(1, dtype=torch.int32, device=dev),
                              info=torch.zeros(1, dtype=torch.int32, device=dev),
                              piv=torch.zeros(NB, dtype=torch.int32, device=dev), rows=ld))
        if max(r["rows"] for r in ranks) > 256 * half:
            print(f"k={k}: {max(r['rows'] for r in ranks)} rows per rank exceed {half} CUs x 256 -- skipped")
            continue
        two = [_Xc(0, 2, bases[:2], slot, dev), _Xc(1, 2, bases[:2], slot, dev)]
        solo = _Xc(0, 1, bases[2:3], slot, dev)

        def run(which, xcs, streams, maxwg):
            lib.dpl_lu_dist_set_maxwg(maxwg)
            for q in which:
                ranks[q]["pv"].copy_(ranks[q]["buf0"])
                ranks[q]["info"].zero_()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for q, xc, st in zip(which, xcs, streams):
                r = ranks[q]
                with torch.cuda.stream(st):
                    r["plu"].run(r["piv"], r["ws"], r["cnt"], r["info"], 0, xc)
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) * 1e3
        res = {}
        for name, which, xcs, sts, mw in (("two", [0, 1], two, [sA, sB], half), ("one", [0], [solo], [sA], half),
                                          ("full", [0], [solo], [sF], 0)):
            ts = [run(which, xcs, sts, mw) for _ in range(4)]
            res[name] = min(ts[1:])
            if name == "two":
                p0, p1 = ranks[0]["piv"].cpu().numpy(), ranks[1]["piv"].cpu().numpy()
                inf = [int(r["info"]) for r in ranks]
                ok = (p0 == p1).all() and (p0 == ref_piv[:NB]).all() and inf == [0, 0]
                res["ok"] = bool(ok)
        lib.dpl_lu_dist_set_maxwg(0)
        xl = (res["two"] - res["one"]) / NB * 1e3
        print(f"k={k:4d} rows/rank {ranks[0]['rows']:6d}/{ranks[1]['rows']:6d}: two {res['two']:7.2f} ms  one "
              f"{res['one']:7.2f} ms  full {res['full']:7.2f} ms  -> per column: two {res['two'] / NB * 1e3:5.2f} "
              f"one {res['one'] / NB * 1e3:5.2f} full {res['full'] / NB * 1e3:5.2f} us; xlat = {xl:5.2f} us; "
              f"pivots == LAPACK on both ranks: {res['ok']}", flush=True)
    for b in bases:
        lib.dpl_xchg_free(ctypes.c_void_p(b))


if __name__ == "__main__":
    main()
