"""Multi-rank DirectSort on CPU: world_size 2 over gloo.

The bench shards the comparator batches of constructRank and the index-check
batches of rotationIndexCheckN over ranks (batch b -> rank b % world) and sums
the partial ciphertexts with one all-reduce each (u64 sum, then mod q) --
DESIGN.md §7.  Here the same protocol runs through the oracle's allreduce hook
with torch.distributed (gloo) as the transport, and the sharded result must be
bit-identical to the unsharded one (reference behaviour: src/sort_algo.h:
182-214 runs the batches serially; sharding must not change the answer).
The GPU engine implements the identical hook (fhe_direct_sort allreduce
callback / RCCL); tests/test_gpu_parity.py checks it against this oracle.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import pyoracle as O

N = 64      # ring 2^11: 4 comparator batches, 4 index-check batches
LOGN = 11


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _gloo_allreduce(buf_ptr, count, _user):
    import ctypes as C
    import torch
    arr = np.ctypeslib.as_array(C.cast(buf_ptr, C.POINTER(C.c_uint64)), shape=(count,))
    t = torch.from_numpy(arr.view(np.int64).copy())
    dist.all_reduce(t, op=dist.ReduceOp.SUM)  # two's-complement wrap == u64 add mod 2^64
    arr[:] = t.numpy().view(np.uint64)


def _worker(rank, world, port, outdir):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    os.environ['OMP_NUM_THREADS'] = '2'
    dist.init_process_group('gloo', rank=rank, world_size=world)
    depth, rots = O.size_parameters(N)
    c = O.Context(LOGN, depth, 40, 60, 3, seed=7)
    c.gen_rotation_keys(rots)
    x = np.random.default_rng(64).permutation(N) / N
    ct = c.encrypt(x, N)
    out = c.direct_sort(ct, N, rots, (3, 3, 2), shard=(rank, world), allreduce=_gloo_allreduce)
    np.save(os.path.join(outdir, f'rank{rank}.npy'), out.data())
    if rank == 0:
        ref = c.direct_sort(ct, N, rots, (3, 3, 2))
        np.save(os.path.join(outdir, 'unsharded.npy'), ref.data())
        np.save(os.path.join(outdir, 'decrypted.npy'), c.decrypt(out))
        np.save(os.path.join(outdir, 'x.npy'), x)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.slow
def test_sharded_direct_sort_world2_matches_unsharded(tmp_path):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method='spawn')
    r0 = np.load(tmp_path / 'rank0.npy')
    r1 = np.load(tmp_path / 'rank1.npy')
    ref = np.load(tmp_path / 'unsharded.npy')
    assert np.array_equal(r0, r1), 'ranks disagree after the all-reduce'
    assert np.array_equal(r0, ref), 'sharded result differs from the unsharded sort'
    x = np.load(tmp_path / 'x.npy')
    y = np.load(tmp_path / 'decrypted.npy')
    assert np.max(np.abs(y - np.sort(x))) < 0.01
