"""Multi-rank DirectSort and MEHP24 sortLargeArrayFG on CPU: world_size 2 over gloo.

The bench shards the comparator batches of constructRank and the index-check
batches of rotationIndexCheckN over ranks (batch b -> rank b % world) and sums
the partial ciphertexts with one all-reduce each (u64 sum, then mod q) --
DESIGN.md §7.  Here the same protocol runs through the oracle's allreduce hook
with torch.distributed (gloo) as the transport, and the sharded result must be
bit-identical to the unsharded one (reference behaviour: src/sort_algo.h:
182-214 runs the batches serially; sharding must not change the answer).
MEHP24 shards its pair compares and indicators the same way (item i on rank
i % world, partial Cv / Ch / subSorted sums all-reduced).
The GPU engine implements the identical hook (fhe_direct_sort allreduce
callback / RCCL); tests/test_gpu_parity.py checks it against this oracle.
"""
import json
import os
import warnings
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


def _input(c, kind):
    """DirectSort N=64, or MEHP24 sortLargeArrayFG of 16 values in parts of 4
    (10 pair compares, 16 indicators -- mehp24_sort.cpp:477-514, 574-594)."""
    n = N if kind == 'direct' else 16
    x = np.random.default_rng(n).permutation(n) / n
    return x, c.encrypt(x, n)


def _run(c, kind, ct, shard=(0, 1), allreduce=None):
    if kind == 'direct':
        depth, rots = O.size_parameters(N)
        return c.direct_sort(ct, N, rots, (3, 3, 2), shard=shard, allreduce=allreduce)
    return c.mehp24_sort(ct, 16, (3, 2, 2), 2, 2, 4, shard=shard, allreduce=allreduce)


def _context(kind):
    if kind == 'direct':
        depth, rots = O.size_parameters(N)
    else:
        depth, rots = 35, O.mehp24_rotation_indices(16, 4)
    c = O.Context(LOGN, depth, 40, 60, 3, seed=7)
    c.gen_rotation_keys(rots)
    return c


def _worker(rank, world, port, outdir, kind):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    # the oracle is OpenMP: split the host's cores between the ranks
    os.environ['OMP_NUM_THREADS'] = str(max(1, (os.cpu_count() or 2) // world))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    c = _context(kind)
    x, ct = _input(c, kind)
    out = _run(c, kind, ct, shard=(rank, world), allreduce=_gloo_allreduce)
    np.save(os.path.join(outdir, f'rank{rank}.npy'), out.data())
    if rank == 0:
        ref = _run(c, kind, ct)
        np.save(os.path.join(outdir, 'unsharded.npy'), ref.data())
        np.save(os.path.join(outdir, 'decrypted.npy'), c.decrypt(out))
        np.save(os.path.join(outdir, 'x.npy'), x)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.slow
@pytest.mark.parametrize('kind', ['direct', 'mehp24'])
def test_sharded_sort_world2_matches_unsharded(tmp_path, kind):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), kind), nprocs=world, join=True,
                       start_method='spawn')
    r0 = np.load(tmp_path / 'rank0.npy')
    r1 = np.load(tmp_path / 'rank1.npy')
    ref = np.load(tmp_path / 'unsharded.npy')
    assert np.array_equal(r0, r1), 'ranks disagree after the all-reduce'
    assert np.array_equal(r0, ref), 'sharded result differs from the unsharded sort'
    x = np.load(tmp_path / 'x.npy')
    y = np.load(tmp_path / 'decrypted.npy')[:len(x)]
    assert np.max(np.abs(y - np.sort(x))) < 0.01


# ---- all-reduce protocol checks: overflow bound, header
# consistency, errors raised inside the hook.  One process; the hook plays the
# other ranks.

def _one_rank_direct():
    c = _context('direct')
    x, ct = _input(c, 'direct')
    return c, ct


def test_world_beyond_u64_bound_is_refused():
    """17 ranks x a 60-bit q0 could wrap the u64 sum of residues: refused."""
    c, ct = _one_rank_direct()
    with pytest.raises(RuntimeError, match='overflow'):
        _run(c, 'direct', ct, shard=(0, 17), allreduce=lambda p, n, u: None)


def test_mismatched_partial_levels_fail_cleanly():
    """A peer whose partial sits at another level makes every rank fail with
    the same error before the data all-reduce (no mismatched collectives)."""
    import ctypes as C
    c, ct = _one_rank_direct()
    calls = []

    def peer_at_other_level(ptr, count, _user):
        arr = np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint64)), shape=(count,))
        calls.append(int(count))
        if count == 4 and arr[0] == 1:  # header of a present partial: add a peer one level up
            l1 = int(arr[1]) + 1
            arr[0] += 1
            arr[1] += l1
            arr[2] += l1 * l1
            arr[3] += int(arr[3]) - 1
    with pytest.raises(RuntimeError, match='differ in level'):
        _run(c, 'direct', ct, shard=(0, 2), allreduce=peer_at_other_level)
    assert calls and all(n == 4 for n in calls), 'the data all-reduce must not start'


def test_exception_in_hook_propagates():
    c, ct = _one_rank_direct()

    class Boom(Exception):
        pass

    def failing(ptr, count, _user):
        raise Boom('transport down')
    with pytest.raises(Boom):
        _run(c, 'direct', ct, shard=(0, 2), allreduce=failing)


# ------------------------------------------------- bench.py multi-rank launch
BENCH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'bench.py')


def _bench(args, timeout=180, env=None):
    import subprocess
    import sys
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout,
                          env=env)


def _json_line(out):
    import json
    lines = [ln for ln in out.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.parametrize('world', [2, 4])
def test_bench_self_launch_rendezvous(world):
    """`python bench.py --gpus N` with no launcher starts its N ranks itself
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set per child, 127.0.0.1 and a
    free port), the ranks meet over gloo, and rank 0 alone prints one JSON line:
    the driver's 1-GPU command shape, run with --gpus N."""
    r = _bench(['--gpus', str(world), '--rendezvous-check'])
    assert r.returncode == 0, r.stderr[-2000:]
    j = _json_line(r.stdout)
    assert j['world'] == world and j['max_rank'] == world - 1 and j['ranks_counted'] == world
    assert j['launcher'] == 'bench.py self-launch'


def test_bench_torchrun_launch_still_works():
    import subprocess
    import sys
    with socket.socket() as so:
        so.bind(('127.0.0.1', 0))
        port = so.getsockname()[1]
    r = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
                        '--master-addr', '127.0.0.1', '--master-port', str(port), BENCH, '--gpus', '2',
                        '--rendezvous-check'], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    j = _json_line(r.stdout)
    assert j['world'] == 2 and j['launcher'] == 'torchrun'


def test_bench_self_launch_failing_rank_ends_the_job():
    """A rank that fails (here: no GPU in this container) must not leave the
    other ranks waiting in a collective: the launcher stops them and returns
    the failure's exit code, quickly."""
    import time
    t = time.time()
    r = _bench(['--gpus', '2', '--steps', '1', '--warmup', '0', '--no-cpu-baseline', '--no-roofline'], timeout=170)
    assert r.returncode != 0
    assert time.time() - t < 160
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith('{')]


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location('bench_under_test', BENCH)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize('world,ndev,local,want', [
    (1, 8, 1, 'none'),     # one rank: no exchange
    (8, 8, 8, 'rccl'),     # the driver's 8-GPU node: one GPU per rank
    (2, 2, 2, 'rccl'),
    (4, 8, 4, 'rccl'),     # fewer ranks than GPUs
    (2, 1, 2, 'gloo'),     # rehearsal: two ranks share one GPU (RCCL refuses duplicate devices)
    (8, 1, 8, 'gloo'),
    (16, 8, 16, 'gloo'),
    (2, 0, 2, 'rccl'),     # devices not probed: trust the launcher
])
def test_bench_collective_selection(world, ndev, local, want):
    """bench.py uses RCCL exactly when every local rank has a GPU of its own,
    and the host + gloo exchange otherwise (verdict r3 item 6)."""
    assert _bench_module().collective_for(world, ndev, local) == want


def test_bench_compute_collective_split():
    """rank_compute_ms / allreduce_ms: each rank's timed wall minus the engine's
    exchange time, max over ranks (a stub context and a one-rank Dist)."""
    m = _bench_module()

    class Ctx:
        def collective_stats(self):
            return {'allreduce_s': 0.25, 'allreduce_calls': 4}

    d = m.Dist(1, probe_devices=False)
    s = m.collective_split(Ctx(), d, 2.0, 2)
    assert s == {'rank_compute_ms': 875.0, 'allreduce_ms': 125.0, 'allreduce_calls_per_step': 2.0}


def test_bench_phase_rows_split_from_kernels():
    """roofline.phases: the clock's 'phase:' rows (MEHP24's sortFG phases) leave the
    per-kernel table untouched -- kernel time and bytes still sum over the kernel
    rows only -- and each phase gets its share and kernel / op-level byte ratio"""
    m = _bench_module()
    stats = {'k_a': {'launches': 2, 'ms': 3.0, 'bytes': 6e9}, 'k_b@modup': {'launches': 1, 'ms': 1.0, 'bytes': 2e9},
             'phase:compare': {'launches': 2, 'ms': 3.0, 'bytes': 6e9, 'op_bytes': 2e9},
             'phase:indicator': {'launches': 1, 'ms': 1.0, 'bytes': 2e9, 'op_bytes': 0.0}}
    k, ph = m.split_phase_rows(stats)
    assert set(k) == {'k_a', 'k_b@modup'} and set(ph) == {'compare', 'indicator'}
    total = sum(v['ms'] for v in k.values())
    t = m.phase_table(ph, total)
    assert list(t) == ['compare', 'indicator']
    assert t['compare']['share'] == 0.75 and t['compare']['kernel_over_op_bytes'] == 3.0
    assert t['compare']['GBps'] == 2000.0 and t['indicator']['kernel_over_op_bytes'] is None


def test_bench_limiter_rule():
    """roofline.limiter (verdicts r3 / r4): a kernel at >= 0.85 of the achievable
    in-place HBM rate is 'hbm'; at >= 0.85 of the measured VALU throughput
    'valu' whatever its waits; 'memory latency' needs >= 0.3 of the wave cycles
    in s_waitcnt and at least its issue stalls -- streaming kernels included
    (k_mul_plain_sum at 0.63 of peak, 0.78 waiting); below both roofs with more
    issue stalls than waits it is 'issue latency' at the compiler's occupancy,
    not 'valu' (r4's headline row pass at valu_frac 0.66)"""
    m = _bench_module()
    lim = lambda *a, **k: m.limiter_of(*a, hbm_ach=0.79, **k)
    assert lim('k_lt_inner<3>', 0.50, {'valu_frac': 0.98, 'wave_cycle_split': {'waitcnt': 0.5, 'issue_stall': 0.2}}) == 'valu'
    assert lim('k_ntt_inv_row<false, false>', 0.20,
               {'valu_frac': 0.32, 'wave_cycle_split': {'waitcnt': 0.52, 'issue_stall': 0.21}}) == 'memory latency'
    assert lim('k_ntt_fwd_row<3, true, true>', 0.61,
               {'valu_frac': 0.65, 'wave_cycle_split': {'waitcnt': 0.23, 'issue_stall': 0.57}},
               4) == 'issue latency (4 waves/SIMD)'
    assert lim('k_mul_plain_sum', 0.63,
               {'valu_frac': 0.27, 'wave_cycle_split': {'waitcnt': 0.78, 'issue_stall': 0.17}}) == 'memory latency'
    assert lim('k_ntt_fwd<8, 4, true, 0, true>', 0.70, {'valu_frac': 0.5}) == 'hbm'
    assert lim('k_add', 0.75, {}) == 'hbm'
    assert 0.5 < m.achievable_hbm_frac() <= 1.0


def test_bench_hbm_ceiling_is_the_best_measured_copy():
    """roofline.hbm_achievable_frac (verdict r5 item 3) is the fastest pattern of
    the committed probe (profiles/r6_rates: the guide's grid-stride 16-B copy,
    100 launches per pattern, two passes), not the best 8-B in-place pattern; the
    headline's 'hbm' label needs >= 0.85 of it."""
    m = _bench_module()
    rows = []
    for name in ('row_pattern.jsonl', 'row_pattern_2.jsonl'):
        with open(os.path.join(os.path.dirname(BENCH), 'profiles', 'r6_rates', name)) as f:
            rows += [json.loads(l) for l in f if l.strip()]
    assert any(r['pattern'].startswith('copy16_gs') for r in rows)
    best = max(r['frac'] for r in rows)
    assert m.achievable_hbm_frac() == best
    assert best >= max(r['frac'] for r in rows if r['pattern'].startswith('copy16_gs'))
    assert m.limiter_of('k', 0.84 * best, {'valu_frac': 0.2, 'wave_cycle_split': {'waitcnt': 0.1, 'issue_stall': 0.5}},
                        3) == 'issue latency (3 waves/SIMD)'
    assert m.limiter_of('k', 0.86 * best, {}) == 'hbm'


def test_counter_tables_are_refused_for_another_library(tmp_path, monkeypatch):
    """The PMC / SQ tables in profiles/ carry the SHA-256 of the library they were
    collected on; bench.py reports their traffic and VALU figures only for that
    library.  A committed table that does not match the in-tree build only WARNS
    here (measurement provenance, not correctness: bench.py then reports those
    figures as null until the next closing profile; FHE_STRICT_TABLES=1 makes it
    fail), and a table stamped with another hash is refused with the reason."""
    m = _bench_module()
    stale = []
    if os.path.exists(m.F.LIB_PATH):
        for name in ('pmc_traffic.json', 'pmc_sq.json', 'pmc_traffic_mehp24.json', 'pmc_sq_mehp24.json',
                     'pmc_traffic_kway.json', 'pmc_sq_kway.json'):
            t, src = m.load_table(name)
            if t is None:  # measurement provenance, not correctness (advisor r4): say so, do not fail
                stale.append(src)
    if stale:
        msg = ('committed counter tables do not match the in-tree library (bench.py reports their '
               'figures as null until the next closing profile): ' + '; '.join(stale))
        if os.environ.get('FHE_STRICT_TABLES') == '1':
            pytest.fail(msg)
        warnings.warn(msg)
    (tmp_path / 'profiles').mkdir()
    (tmp_path / 'profiles' / 'pmc_x.json').write_text(json.dumps({'_meta': {'lib_sha256': '0' * 64}, 'k_add': {}}))
    monkeypatch.setattr(m, 'REPO', str(tmp_path))
    t, src = m.load_table('pmc_x.json')
    assert t is None and 'stale' in src


def test_committed_tables_cover_the_profiled_kernels():
    """Every kernel of the closing profile's sort-only trace that takes >= 1% of the
    sort (profiles/r6_final/region_kernel_stats.csv) has a row in the committed
    instruction-mix table (profiles/valu_mix.json, the roofline's VALU pricing) and
    in the SQ counter table, so the bench line's valu_frac / limiter are defined for
    the kernels that matter -- the newer kernels (k_leaf_sums_fold, k_tensor_lin,
    k_modup_fold, round 6's k_moddown_rescale_fp) included."""
    import csv
    import re
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    stats = os.path.join(repo, 'profiles', 'r6_final', 'region_kernel_stats.csv')
    if not os.path.exists(stats):
        pytest.skip('no closing profile committed')
    rows = list(csv.DictReader(open(stats)))
    total = sum(float(r['TotalDurationNs']) for r in rows)
    mix = json.load(open(os.path.join(repo, 'profiles', 'valu_mix.json')))
    sq = json.load(open(os.path.join(repo, 'profiles', 'pmc_sq.json')))
    missing = []
    for r in rows:
        if float(r['TotalDurationNs']) < 0.01 * total:
            continue
        m = re.search(r'(k_[a-z0-9_]+(<[^>]*>)?)\(', r['Name'])
        name = m.group(1) if m else r['Name']
        if name not in mix or name not in sq:
            missing.append(name)
    assert not missing, missing
    assert any(k.startswith('k_leaf_sums_fold<') for k in mix)
    assert any(k.startswith('k_tensor_lin<') for k in mix)
    assert any(k.startswith('k_moddown_rescale_fp<') for k in mix) and any(k.startswith('k_moddown_rescale_fp<') for k in sq)
