"""Probe: can two ranks share the one GPU of a gpurun box over the "nccl" (RCCL) backend?  Each rank all-gathers a
rank-stamped tensor; prints the result or the error.  (RCCL, like NCCL, may refuse two ranks on one device.)

    timeout -k 10 120 python tools/rccl_probe.py
"""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        x = torch.full((4,), float(rank + 1), device=dev)
        out = torch.empty(world * 4, device=dev)
        dist.all_gather_into_tensor(out, x)
        torch.cuda.synchronize()
        q.put((rank, "ok", out.cpu().tolist()))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 - the probe reports whatever RCCL raises
        q.put((rank, "error", repr(e)[:400]))


if __name__ == "__main__":
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, world, 29533, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=100) for _ in ps]
    for p in ps:
        p.join(timeout=30)
    for r in sorted(res):
        print(r)
    sys.exit(0 if all(r[1] == "ok" for r in res) else 1)
