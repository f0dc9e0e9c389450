"""Does RCCL run two ranks on ONE GPU (the 1-GPU boxes' only way to exercise the N > 1 RCCL path)? Two processes,
backend nccl, both on cuda:0: an all_reduce of a 25 MB bucket and a barrier. Prints the result or the error.

    python scripts/rccl_two_rank_probe.py
"""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    try:
        torch.cuda.set_device(0)
        dist.init_process_group('nccl', rank=rank, world_size=world, device_id=torch.device('cuda', 0))
        x = torch.full((25 * 1024 * 1024 // 4,), float(rank + 1), device='cuda')
        dist.all_reduce(x)
        torch.cuda.synchronize()
        dist.barrier()
        q.put((rank, 'ok', float(x[0].item())))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, 'error', repr(e)[:300]))


def main():
    world, port = 2, 29611
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=90) for _ in range(world)]
    for p in ps:
        p.join(timeout=30)
    for r in sorted(res):
        print(r)
    sys.exit(0 if all(r[1] == 'ok' and r[2] == 3.0 for r in res) else 1)


if __name__ == '__main__':
    main()
