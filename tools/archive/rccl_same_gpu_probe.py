"""Probe: can two ranks share one GPU under RCCL? (expected: RCCL refuses duplicates)."""
import os, sys, datetime
import torch
import torch.multiprocessing as mp

def run(rank, size, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(size))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=size, timeout=datetime.timedelta(seconds=30))
    x = torch.ones(4, device="cuda") * (rank + 1)
    dist.all_reduce(x)
    torch.cuda.synchronize()
    print(rank, x.tolist(), flush=True)
    dist.destroy_process_group()

if __name__ == "__main__":
    import socket
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    mp.spawn(run, args=(2, port), nprocs=2)
