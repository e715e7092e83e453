"""Sharded DirectSort and MEHP24 sortLargeArrayFG on the GPU engine, two ranks on one MI355X.

Each rank owns a context on device 0 (deterministic key generation: identical
keys and encryptions), runs batches b with b % 2 == rank, and sums the partial
ciphertexts through the fhe_direct_sort all-reduce callback (here: device ->
host copy, gloo all_reduce, host -> device; on a multi-GPU node the bench uses
RCCL through fhe_comm_init instead).  The sharded result must equal the
unsharded one word for word.
"""
import ctypes as C
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, LOGN = 64, 11  # 4 comparator batches + 4 index-check batches


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, outdir, kind):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    import torch
    import torch.distributed as dist
    import fhesort as F
    dist.init_process_group('gloo', rank=rank, world_size=world)
    hip = C.CDLL('libamdhip64.so')
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    D2H, H2D = 2, 1

    def allreduce(ptr, count, _user):
        buf = np.empty(count, dtype=np.uint64)
        assert hip.hipMemcpy(buf.ctypes.data, C.cast(ptr, C.c_void_p), count * 8, D2H) == 0
        t = torch.from_numpy(buf.view(np.int64))
        dist.all_reduce(t, op=dist.ReduceOp.SUM)  # two's-complement wrap == u64 add
        assert hip.hipMemcpy(C.cast(ptr, C.c_void_p), buf.ctypes.data, count * 8, H2D) == 0

    if kind == 'direct':
        depth, rots = F.size_parameters(N)
        n = N
    else:  # MEHP24 sortLargeArrayFG, 16 values in parts of 4: 10 pair compares, 16 indicators
        depth, rots, n = 35, F.mehp24_rotation_indices(16, 4), 16
    ctx = F.Context(LOGN, depth, 40, 60, 3, seed=31)
    ctx.gen_rotation_keys(rots)
    ctx.set_sort_stack(2)
    x = np.random.default_rng(5).permutation(n) / n
    ct = ctx.encrypt(x, n)

    def run(**kw):
        if kind == 'direct':
            return ctx.direct_sort(ct, N, rots, (3, 3, 2), **kw)
        return ctx.mehp24_sort(ct, 16, (3, 2, 2), 2, 2, 4, **kw)
    out = run(shard=(rank, world), allreduce=allreduce)
    np.save(os.path.join(outdir, f'rank{rank}.npy'), out.data())
    if rank == 0:
        ref = run()
        np.save(os.path.join(outdir, 'ref.npy'), ref.data())
        np.save(os.path.join(outdir, 'dec.npy'), ctx.decrypt(out)[:n])
        np.save(os.path.join(outdir, 'x.npy'), x)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('kind', ['direct', 'mehp24'])
def test_two_ranks_one_gpu_match_unsharded(tmp_path, kind):
    import torch.multiprocessing as mp
    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path), kind), nprocs=2, join=True,
                       start_method='spawn')
    r0, r1, ref = (np.load(tmp_path / f) for f in ('rank0.npy', 'rank1.npy', 'ref.npy'))
    assert np.array_equal(r0, r1), 'ranks disagree after the all-reduce'
    assert np.array_equal(r0, ref), 'sharded GPU sort differs from the unsharded one'
    x, y = np.load(tmp_path / 'x.npy'), np.load(tmp_path / 'dec.npy')
    assert np.max(np.abs(y - np.sort(x))) < 0.01
