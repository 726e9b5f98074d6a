"""Can two ranks share one GPU over RCCL (backend "nccl")?  If yes, the RCCL-only branches of the
transport (parallel.p2p comm-stream path, all_gather_into_tensor, batch_isend_irecv) can be rehearsed on
a one-GPU box.  Prints RCCL_SAME_GPU ok/fail with the error."""
import os
import sys

import torch
import torch.distributed as dist


def main():
    torch.cuda.set_device(0)
    try:
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
        r = dist.get_rank()
        t = torch.full((4,), float(r + 1), device="cuda")
        dist.all_reduce(t)
        out = torch.zeros(2 * 4, device="cuda")
        dist.all_gather_into_tensor(out, t)
        peer = 1 - r
        s, q = torch.full((3,), float(r), device="cuda"), torch.zeros(3, device="cuda")
        ops = [dist.P2POp(dist.isend, s, peer), dist.P2POp(dist.irecv, q, peer)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        torch.cuda.synchronize()
        ok = float(t[0]) == 3.0 and float(q[0]) == float(peer)
        print(f"RCCL_SAME_GPU rank {r}: {'ok' if ok else 'wrong values'} allreduce={t.tolist()} p2p={q.tolist()}",
              flush=True)
        dist.destroy_process_group()
        sys.exit(0 if ok else 1)
    except Exception as e:  # noqa: BLE001
        print(f"RCCL_SAME_GPU rank {os.environ.get('RANK')}: fail {type(e).__name__}: {e}", flush=True)
        sys.exit(3)


if __name__ == "__main__":
    main()
