"""Shared test helpers: dense references and multi-process (gloo) launcher."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

DTYPES = {"s": torch.float32, "d": torch.float64, "c": torch.complex64, "z": torch.complex128}


def tol(dtype):
    return 2e-3 if dtype in (torch.float32, torch.complex64) else 1e-10


def rel_err(x, ref):
    x = x.to(torch.complex128 if x.is_complex() or ref.is_complex() else torch.float64)
    ref = ref.to(x.dtype)
    d = (x - ref).abs().max().item()
    s = ref.abs().max().item() or 1.0
    return d / s


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _TensorBox:
    def __init__(self, arr):
        self.arr = arr


def _plain(x, to_np=True):
    """Results cross the process boundary by value: tensors as numpy arrays (a tensor sent through
    an mp.Queue is shared by file descriptor and races with the exiting child)."""
    if to_np and isinstance(x, torch.Tensor):
        return _TensorBox(x.detach().cpu().numpy().copy())
    if not to_np and isinstance(x, _TensorBox):
        return torch.from_numpy(x.arr)
    if isinstance(x, (list, tuple)):
        return type(x)(_plain(v, to_np) for v in x)
    if isinstance(x, dict):
        return {k: _plain(v, to_np) for k, v in x.items()}
    return x


def _worker(rank, world, port, fn, args, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r = fn(rank, world, *args)
        q.put((rank, "ok", _plain(r)))
    except Exception as e:  # pragma: no cover - reported to parent
        import traceback
        q.put((rank, "err", traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def run_distributed(fn, world, *args, timeout=240):
    """Run fn(rank, world, *args) on `world` gloo CPU ranks; returns {rank: result}."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            rank, status, r = q.get(timeout=timeout)
            if status != "ok":
                raise RuntimeError(f"rank {rank} failed:\n{r}")
            out[rank] = _plain(r, to_np=False)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return out
