"""Probe the RCCL path (fhe_comm_init + fhe_ct_allreduce) with two ranks.

Each rank builds the same small context (deterministic keys), encrypts the
same vector, all-reduces the ciphertext through RCCL and decrypts: the result
must be 2x the input.  On a one-GPU box both ranks sit on device 0, which
RCCL may refuse (duplicate device); the probe then reports the error code
that fhe_comm_init returned instead of crashing.

  python scripts/rccl_probe.py [--world 2]
"""
import argparse
import os
import socket
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'fhe-sorting_amd'))


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, ndev):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    import torch.distributed as dist
    import fhesort as F
    dist.init_process_group('gloo', rank=rank, world_size=world)
    ctx = F.Context(11, 4, 40, 60, 3, seed=7, device=rank % ndev)
    x = np.linspace(-0.5, 0.5, 64)
    ct = ctx.encrypt(x, 64)
    obj = [F.Context.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    try:
        ctx.comm_init(obj[0], rank, world)
    except Exception as e:  # noqa: BLE001 - report and leave
        print(f'rank {rank}: fhe_comm_init failed: {e}', flush=True)
        dist.barrier()
        return
    ctx.ct_allreduce(ct)
    y = ctx.decrypt(ct)[:64]
    err = float(np.max(np.abs(y - world * x)))
    print(f'rank {rank}: RCCL all-reduce of {world} ciphertexts, max |dec - {world}x| = {err:.3e}', flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--world', type=int, default=2)
    a = ap.parse_args()
    import torch
    import torch.multiprocessing as mp
    ndev = max(1, torch.cuda.device_count())
    mp.start_processes(_worker, args=(a.world, _free_port(), ndev), nprocs=a.world, join=True, start_method='spawn')


if __name__ == '__main__':
    main()
