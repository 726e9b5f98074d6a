"""The round-5 w4 anomaly (bench.py race: distributed DTR 40 ms, timed steps 269 ms; r6_b2: 41 ms vs 199.5 ms) with
four ranks sharing ONE GPU: time the distributed DTR (a) fresh, (b) after the rank has also used its other HIP streams
(the stream engine's panel / update / aux streams and one RCCL-free gloo round), (c) again after a device-wide
synchronize.  If (b) jumps, the slowdown is hardware-queue oversubscription between the four processes (the GPU
time-slices their queues; a persistent kernel that must run beside its peers' advances only while all four are
mapped) -- not the DTR: one process per GPU has no such sharing.

  DPLASMA_DIST_BACKEND=gloo DPLASMA_DTR_WG=64 python -m torch.distributed.run --nproc-per-node 4 \\
      --master-addr 127.0.0.1 tools/gpu/dtr_w4_queues.py [N]"""
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    import dplasma_amd as dp
    from dplasma_amd.models import potrf_dtr_dist
    ctx = dp.init(P=dist.get_world_size())
    A = dp.block_cyclic(ctx, torch.float64, 512, 512, N, N)
    dp.plghe(ctx, float(N), dp.dplasmaLower, A, 3872)
    A0 = A.data.clone()
    tpd = potrf_dtr_dist.potrf_dtr_dist_New(ctx, dp.dplasmaLower, A)

    def timed(tp, n=3):
        out = []
        for _ in range(n):
            A.data.copy_(A0)
            tp.info.zero_()
            ctx.sync()
            ctx.barrier()
            t0 = time.perf_counter()
            tp.run(ctx)
            ctx.sync()
            out.append((time.perf_counter() - t0) * 1e3)
            tp.complete(ctx)
        return out
    a = timed(tpd)
    # touch the context's other streams with real work (what the stream engine's run does)
    for name in ("panel", "update", "aux"):
        with torch.cuda.stream(ctx.streams[name]):
            torch.ones(1 << 20, device=ctx.device).sum()
    ctx.sync()
    b = timed(tpd)
    torch.cuda.synchronize()
    c = timed(tpd)
    # (d) after one run of the stream engine (what bench.py's race does before the timed steps)
    os.environ["DPLASMA_POTRF_ENGINE"] = "stream"
    tps = dp.potrf_New(ctx, dp.dplasmaLower, A)
    s_ = timed(tps, 1)
    d = timed(tpd)
    # (e) the bench's timed step: + barrier + sync after the run, inside the timed region
    e = []
    for _ in range(3):
        A.data.copy_(A0)
        tpd.info.zero_()
        ctx.sync()
        ctx.barrier()
        ctx.sync()
        t0 = time.perf_counter()
        tpd.run(ctx)
        ctx.sync()
        ctx.barrier()
        ctx.sync()
        e.append((time.perf_counter() - t0) * 1e3)
    tpd.complete(ctx)
    if ctx.rank == 0:
        print(f"w{ctx.world} N={N}: fresh {['%.1f' % x for x in a]} ms | after the other streams ran "
              f"{['%.1f' % x for x in b]} | again {['%.1f' % x for x in c]} | stream engine {s_[0]:.1f} ms, then "
              f"{['%.1f' % x for x in d]} | bench step shape {['%.1f' % x for x in e]}", flush=True)
    potrf_dtr_dist.release_all()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
