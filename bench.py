#!/usr/bin/env python3
"""Benchmark: encrypted rank sort (DirectSort) on MI355X.

Workload (BASELINE.json metric): DirectSort of N=1024 reals at ring dimension
2^16, multiplicative depth 39 (40 Q primes: 60-bit q0 + the reference's 40-bit
scaling primes, K special primes, dnum=3; OpenFHE's Paterson-Stockmeyer split),
161 rotation keys, CompositeSign(3,5,2) -- the reference's DirectSortTest
configuration for N=1024 (tests/DirectSortTest.cpp:104-112,
src/sort_algo.h:147-165).  One step = one full sort() of an encrypted input
already resident in HBM (constructRank + rotationIndexCheckN); keys, the
input encryption and the public plaintext masks are produced before timing.

Multi-GPU (one process per GPU: `python bench.py --gpus N` starts the N ranks
itself, or run it under torchrun): the 32 comparator batches of
constructRank and the 32 index-check batches of rotationIndexCheckN are
sharded over ranks (batch b -> rank b % world); the partial ranks/outputs are
summed by one RCCL all-reduce each (u64 sum + mod q) -- strong scaling.

--workload mehp24: MEHP24 sortLargeArrayFG of N=4096 at ring 2^17 (BASELINE
config 5), pair compares and indicators sharded over ranks.

--workload kway: the k-way sorting network with bootstrapping, k=5, N=3125 at
ring 2^16 (BASELINE config 4; KWaySort235Test's context: depth 40, scale 2^59,
levelBudget {5,5}).  The network is one chain of stages on one ciphertext, so
it does not shard: --gpus N runs N independent replicas (weak scaling).

Output: one JSON line.  value = ciphertext-mults/s (relinearised ct x ct
products, incl. those in the Chebyshev PS, summed over ranks / wall time);
ms_per_step = sort wall time.  Also: roofline of the dominant kernel (HIP
events on the engine stream) and the CPU-oracle baseline (rank 0, every world size).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, 'fhe-sorting_amd'))
# the sharded sort times its partial-sum exchanges (allreduce_ms) only when asked
os.environ.setdefault('FHE_TIME_COLLECTIVES', '1')

import fhesort as F  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
MFMA_SIMDS = 1024           # 256 CUs x 4 SIMDs (MI355X_MICROARCH.md)
PEAK_CLOCK_HZ = 2.4e9      # peak engine clock
N_SIMD = 256 * 4        # 256 CUs x 4 SIMDs
F_CLK = 2.4e9           # peak engine clock (the effective clock under load is lower: valu_frac is a lower bound)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=2)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--workload', choices=('direct', 'mehp24', 'kway'), default='direct',
                    help='direct: DirectSort rank sort (the BASELINE metric); mehp24: MEHP24 sortLargeArrayFG '
                         '(BASELINE config 5, ring 2^17); kway: k-way network with bootstrapping (config 4)')
    ap.add_argument('--kway-k', type=int, default=5)
    ap.add_argument('--kway-m', type=int, default=5)
    ap.add_argument('--n-sort', type=int, default=None, help='values to sort (default 1024; mehp24: 4096)')
    ap.add_argument('--log-n', type=int, default=16)
    ap.add_argument('--seed', type=int, default=20250704)
    ap.add_argument('--scale-bits', type=int, default=40,
                    help="scaling-prime size (the reference's 40, src/sort_algo.h:92,199)")
    ap.add_argument('--ps-split', choices=('openfhe', 'engine'), default='openfhe',
                    help="Paterson-Stockmeyer split: OpenFHE's (the reference's EvalChebyshevSeriesPS; holds the "
                         "0.01 bound at 40 bits) or rounds 1-2's power-of-two split (needs 50 bits at N=1024), "
                         "DESIGN.md §3")
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-roofline', action='store_true', help='skip the instrumented roofline sort (PMC passes)')
    ap.add_argument('--cpu-sample-mults', type=int, default=0, help='override CPU sample size')
    ap.add_argument('--clock-json', default=None, help='write the full per-kernel clock of the roofline sort here')
    ap.add_argument('--dnum', type=int, default=0, help='MEHP24: key-switch digits (0: the parameter table, OpenFHE default 3)')
    ap.add_argument('--lanes', type=int, default=2,
                    help='concurrent batch lanes (forked engines) per GPU (round 4, batched rotations: 2 lanes 589.6 ms, '
                         '3 lanes 604.0, 4 lanes 611.9, 1 lane 613.8; profiles/r4_lanes)')
    ap.add_argument('--stack', type=int, default=32, help='max batches stacked into one ciphertext batch')
    ap.add_argument('--mask-steps', type=int, default=2,
                    help='extra sorts timed with every mask re-encoded per sort (0: skip)')
    ap.add_argument('--rendezvous-check', action='store_true',
                    help='launch/rendezvous only: ranks meet over gloo, exchange a max and a sum, rank 0 prints '
                         'one JSON line (no GPU work; the multi-rank launcher test)')
    return ap.parse_args()


def launched_by_torchrun():
    return 'RANK' in os.environ and 'WORLD_SIZE' in os.environ


def self_launch(a):
    """`python bench.py --gpus N` without a launcher: start N fresh interpreters
    running this script as ranks 0..N-1 (the env torchrun would set: RANK,
    LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, a free
    MASTER_PORT), before this process touches HIP or torch.cuda.  Rank 0 prints
    the JSON line on the inherited stdout; if any rank fails the others are
    stopped and the exit code is the first failure's."""
    import signal
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(('127.0.0.1', 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus),
                   LOCAL_WORLD_SIZE=str(a.gpus), MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      start_new_session=True))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in live:  # a rank that failed leaves the others waiting in a collective
                        try:
                            os.killpg(q.pid, signal.SIGTERM)
                        except ProcessLookupError:
                            pass
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
    return rc if rc >= 0 else 128 - rc


def rendezvous_check(a, d):
    t = time.perf_counter()
    d.barrier()
    mx = d.max(float(d.rank))
    sm = d.sum(1.0)
    d.barrier()
    if d.rank == 0:
        print(json.dumps({'rendezvous': 'ok', 'world': d.world, 'max_rank': mx, 'ranks_counted': sm,
                          'launcher': 'torchrun' if os.environ.get('TORCHELASTIC_RUN_ID') else 'bench.py self-launch'
                          if d.world > 1 else 'none', 'seconds': round(time.perf_counter() - t, 3)}), flush=True)


def sign_cfg(N):  # tests/DirectSortTest.cpp:104-112
    if N <= 16:
        return (3, 2, 2)
    if N <= 128:
        return (3, 3, 2)
    if N <= 512:
        return (3, 4, 2)
    return (3, 5, 2)


def collective_for(world, ndev, local_world):
    """The partial-sum exchange of a sharded run: 'none' for one rank; 'rccl'
    when every local rank has a GPU of its own (ndev 0 = not probed: trust the
    launcher); 'gloo' (host memory) otherwise -- RCCL refuses two ranks on one
    device (rccl.h), so a rehearsal with more ranks than GPUs goes through the host"""
    if world <= 1:
        return 'none'
    return 'rccl' if ndev == 0 or ndev >= local_world else 'gloo'


class ProfRegion:
    """FHE_PROF_REGION=1: empty marker kernels (k_region_begin / k_region_end,
    fhe_region_marker) on the engine stream bracket the timed sorts, so a
    rocprofv3 kernel trace or PMC pass of this run can be cut to the sort alone
    (scripts/pmc_meta.py region filter: key generation, encryption and the
    warmup sort stay out of profiles/r4_*).  Without the variable: nothing."""

    def __init__(self, ctx):
        self.ctx = ctx if os.environ.get('FHE_PROF_REGION') == '1' else None

    def resume(self):
        if self.ctx:
            self.ctx.region_marker(True)

    def pause(self):
        if self.ctx:
            self.ctx.region_marker(False)
            self.ctx.sync()


class Dist:
    def __init__(self, world, probe_devices=True):
        self.world = world
        self.rank = int(os.environ.get('RANK', '0'))
        self.local = int(os.environ.get('LOCAL_RANK', '0'))
        ndev = 0
        if probe_devices:  # one rank per GPU; ranks beyond the visible devices share them (rehearsals only)
            try:
                import torch
                ndev = torch.cuda.device_count()
            except Exception:
                ndev = 0
        self.device = self.local % ndev if ndev > 0 else self.local
        self.collective = collective_for(world, ndev, int(os.environ.get('LOCAL_WORLD_SIZE', world)))
        self.rccl = self.collective == 'rccl'
        self.pg = None
        if world > 1:
            import torch.distributed as dist
            os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
            dist.init_process_group('gloo', rank=self.rank, world_size=world)
            self.dist = dist

    def host_allreduce(self):
        import ctypes as C
        import torch
        hip = C.CDLL('libamdhip64.so')
        hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]

        def fn(ptr, count, _user):
            buf = np.empty(count, dtype=np.uint64)
            if hip.hipMemcpy(buf.ctypes.data, C.cast(ptr, C.c_void_p), count * 8, 2) != 0:
                raise RuntimeError('hipMemcpy D2H failed')
            self.dist.all_reduce(torch.from_numpy(buf.view(np.int64)), op=self.dist.ReduceOp.SUM)
            if hip.hipMemcpy(C.cast(ptr, C.c_void_p), buf.ctypes.data, count * 8, 1) != 0:
                raise RuntimeError('hipMemcpy H2D failed')
        return fn

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def bcast_bytes(self, b):
        if self.world == 1:
            return b
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def max(self, v):
        if self.world == 1:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, v):
        if self.world == 1:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())


def device_sync(ctx):
    ctx.sync()
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    except Exception:
        pass


_LIB_SHA = None


def lib_sha256():
    """SHA-256 of the loaded engine library: the committed PMC tables carry the
    hash of the build they were collected on (scripts/pmc_summary.py --lib), and
    counters of another build are not reported as this one's"""
    global _LIB_SHA
    if _LIB_SHA is None:
        import hashlib
        h = hashlib.sha256()
        with open(F.LIB_PATH, 'rb') as f:
            for chunk in iter(lambda: f.read(1 << 20), b''):
                h.update(chunk)
        _LIB_SHA = h.hexdigest()
    return _LIB_SHA


def load_table(fname):
    """(table, source) of a committed profiles/ table (PMC traffic, SQ counters);
    (None, reason) when absent or collected on a different libfhesort.so"""
    path = os.path.join(REPO, 'profiles', fname)
    if not os.path.exists(path):
        return None, f'profiles/{fname} absent'
    with open(path) as f:
        t = json.load(f)
    meta = t.pop('_meta', {})
    want = lib_sha256()
    if meta.get('lib_sha256') != want:
        return None, (f'profiles/{fname} is stale: collected on libfhesort.so {str(meta.get("lib_sha256"))[:12]}, '
                      f'loaded {want[:12]}')
    return t, f'profiles/{fname}'


def family(name):
    """'k_ntt_fwd<8, 4, true, 0, true>@modup' -> 'k_ntt_fwd'"""
    return name.split('@')[0].split('<')[0]


def table_keys(table, name, by_family):
    if table is None:
        return []
    if by_family:
        return [k for k in table if family(k) == name]
    return [name] if name in table else []


def weighted(table, keys, field):
    n = sum(table[k]['launches'] for k in keys)
    return sum(table[k].get(field, 0) * table[k]['launches'] for k in keys) / n if n else 0.0


def valu_fraction(sq, mix, keys, avg_s):
    """The compute roof: the share of the chip's measured VALU throughput the
    launches use.  valu_frac = SQ_INSTS_VALU per launch (the committed SQ pass
    of the same workload and build, profiles/pmc_sq*.json,
    scripts/pmc_sq_summary.py) x 64 lanes x the seconds one lane-instruction of
    the kernel's instruction mix costs at the measured MI355X rates
    (profiles/valu_mix.json, scripts/valu_mix.py: full-rate 67.5 T, half-rate
    36 T, v_mad_u64_u32 23 T, carry/compare pairs 39 T lane-instructions/s) /
    the live average launch duration.  Near 1: VALU-bound.  Instantiations of
    one family are launch-weighted."""
    keys = [k for k in keys if k in mix and 'SQ_INSTS_VALU' in sq[k]]
    if not keys:
        return {}
    n = sum(sq[k]['launches'] for k in keys)
    valu_s = sum(sq[k]['launches'] * sq[k]['SQ_INSTS_VALU'] * 64 * mix[k]['ps_per_lane_instr'] * 1e-12
                 for k in keys) / n
    wc = weighted(sq, keys, 'SQ_WAVE_CYCLES') or 1
    out = {'valu_frac': round(valu_s / avg_s, 4), 'valu_insts_per_launch': round(weighted(sq, keys, 'SQ_INSTS_VALU')),
           'valu_seconds_per_launch': valu_s,
           'wave_cycle_split': {'waitcnt': round(weighted(sq, keys, 'SQ_WAIT_ANY') / wc, 3),
                                'issue_stall': round(weighted(sq, keys, 'SQ_WAIT_INST_ANY') / wc, 3)}}
    # matrix-core kernels (the i8 sums of products): SQ_VALU_MFMA_BUSY_CYCLES is
    # the MFMA pipe's busy SIMD-cycles per launch (16 per v_mfma_i32_16x16x64_i8);
    # over 1024 SIMDs x the 2.4 GHz peak clock x the live launch duration
    busy = weighted(sq, keys, 'SQ_VALU_MFMA_BUSY_CYCLES')
    if busy > 0:
        out['mfma_frac'] = round(busy / (MFMA_SIMDS * PEAK_CLOCK_HZ * avg_s), 4)
    return out


def achievable_hbm_frac():
    """The best HBM rate a plain copy reaches on an MI355X, as a fraction of the
    8 TB/s peak: the fastest pattern of scripts/row_pattern.hip over both of its
    passes (round 6, profiles/r6_rates/row_pattern*.jsonl) -- the guide's
    grid-stride 16-B copy with 4-8 loads in flight per thread (5.94 TB/s = 0.742
    in the first pass, 0.68 in the second on the same box a second later; the
    guide's own figure is 6.29 TB/s = 0.786), the in-place and the NTT passes' own
    block shapes (0.72 and 0.71 in the first pass).  0.786 when the files are
    absent."""
    rows = []
    for name in ('row_pattern.jsonl', 'row_pattern_2.jsonl'):
        try:
            rows += [json.loads(l) for l in open(os.path.join(REPO, 'profiles', 'r6_rates', name)) if l.strip()]
        except (OSError, ValueError):
            pass
    try:
        return max(r['frac'] for r in rows)
    except (ValueError, KeyError):
        return 0.786


def limiter_of(name, frac, vf, waves=None, hbm_ach=None):
    """What bounds the kernel: 'hbm' at >= 0.85 of the best measured copy rate
    (achievable_hbm_frac(), whatever the kernel); 'valu' at >= 0.85 of the
    measured VALU throughput (whatever its waits); 'memory latency' when the SQ
    pass puts >= 0.3 of its wave cycles in s_waitcnt, at least its issue
    stalls; else 'issue latency (W waves/SIMD)': dependent-instruction stalls at
    the compiler's occupancy W (profiles/valu_mix.json), neither roof reached"""
    ach = achievable_hbm_frac() if hbm_ach is None else hbm_ach
    if frac >= 0.85 * ach:
        return 'hbm'
    if vf.get('valu_frac', 0) >= 0.85:
        return 'valu'
    split = vf.get('wave_cycle_split', {})
    if split.get('waitcnt', 0) >= max(0.3, split.get('issue_stall', 0)):
        return 'memory latency'
    if split.get('issue_stall', 0) > split.get('waitcnt', 0):
        return f'issue latency ({waves} waves/SIMD)' if waves else 'issue latency'
    return 'memory latency'


def kernel_view(name, st, pmc, sq, mix, by_family):
    """frac, traffic and compute roof of one kernel (an exact rocprofv3 symbol, or
    every instantiation of a family) from the live clock + committed tables"""
    avg_s = st['ms'] / st['launches'] * 1e-3
    per_launch = st['bytes'] / st['launches']
    achieved = per_launch / avg_s / 1e9
    frac = achieved / HBM_PEAK_GBS
    pk = table_keys(pmc, name, by_family)
    traffic = round(weighted(pmc, pk, 'hbm_bytes_per_launch')) if pk else None
    vf = valu_fraction(sq, mix, table_keys(sq, name, by_family), avg_s) if sq and mix else {}
    mk = [k for k in table_keys(mix, name, by_family) if 'waves_per_simd' in mix[k]] if mix else []
    waves = min(mix[k]['waves_per_simd'] for k in mk) if mk else None
    return {'kernel': name, 'achieved': round(achieved, 1), 'frac': round(frac, 4), 'traffic': traffic,
            'traffic_ratio': round(traffic / per_launch, 3) if traffic else None,
            'limiter': limiter_of(name, frac, vf, waves), 'waves_per_simd': waves,
            'frac_of_achievable': round(frac / achievable_hbm_frac(), 4), **vf,
            'avg_us': round(avg_s * 1e6, 2), 'launches': st['launches'], 'algorithmic_bytes_per_launch': per_launch}


def split_phase_rows(stats):
    """The live clock's 'phase:<name>' rows -- the same kernels booked again under
    the algorithm phase that launched them (MEHP24: split / replicate / compare /
    rank_sums / indicator / select / recombine), with that phase's SURVEY §8(d)
    op-level bytes -- apart from the per-kernel rows (which alone sum to the sort)"""
    kernels = {k: v for k, v in stats.items() if not k.startswith('phase:')}
    phases = {k[6:]: v for k, v in stats.items() if k.startswith('phase:')}
    return kernels, phases


def phase_table(phase_rows, total_ms):
    """roofline.phases: per phase its kernel time and share, launches, kernel bytes,
    op-level bytes, their ratio and kernel GB/s, longest first"""
    return {n: {'ms': round(v['ms'], 2), 'share': round(v['ms'] / total_ms, 3), 'launches': v['launches'],
                'kernel_bytes': v['bytes'], 'op_bytes': v.get('op_bytes', 0.0),
                'kernel_over_op_bytes': round(v['bytes'] / v['op_bytes'], 2) if v.get('op_bytes') else None,
                'GBps': round(v['bytes'] / (v['ms'] * 1e-3) / 1e9, 1) if v['ms'] else None}
            for n, v in sorted(phase_rows.items(), key=lambda kv: -kv[1]['ms'])}


def roofline(ctx, run_once, dump=None, pmc_file='pmc_traffic.json', sq_file='pmc_sq.json'):
    """Roofline of the dominant kernel, measured live: one more (untimed) sort
    runs with every hot kernel launched through hipExtLaunchKernelGGL with
    start/stop events on the engine stream (the stream it runs on), one lane so
    no other kernel overlaps the measured span.  Two dominance views:
      * the headline (`kernel`, `frac`, ...) is the kernel with the largest total
        time by exact rocprofv3 symbol (template instantiation; the clock's
        caller tags '@modup' are aggregated the way rocprofv3 --stats does), so
        profiles/<run>/run_kernel_stats.csv reproduces it directly;
      * `by_family`: the largest family when a family's instantiations are
        aggregated (e.g. the six k_linear_sum_mfma<KS, NG>).
    achieved = algorithmic bytes per launch / average launch
    duration.  traffic = HBM bytes per launch from the committed rocprofv3 PMC
    passes (FETCH_SIZE x2 on gfx950 + WRITE_SIZE), valu_frac / mfma_frac from
    the committed SQ pass -- both only when collected on the loaded
    libfhesort.so (its SHA-256 is stamped in the table; otherwise null and
    `pmc_source` says why)."""
    with F.KernelClock(ctx) as clk:
        run_once()  # single lane: concurrent lanes would inflate each kernel's event span
    stats = clk.stats
    if dump:
        with open(dump, 'w') as f:
            json.dump(stats, f, indent=1)
    stats, phase_rows = split_phase_rows(stats)
    total_ms = sum(v['ms'] for v in stats.values())
    by_sym, by_fam = {}, {}
    for k, v in stats.items():
        for agg, key in ((by_sym, k.split('@')[0]), (by_fam, family(k))):
            a = agg.setdefault(key, {'ms': 0.0, 'launches': 0, 'bytes': 0.0})
            a['ms'] += v['ms']
            a['launches'] += v['launches']
            a['bytes'] += v['bytes']
    pmc, pmc_src = load_table(pmc_file)
    sq, sq_src = load_table(sq_file)
    mix_path = os.path.join(REPO, 'profiles', 'valu_mix.json')
    mix = json.load(open(mix_path)) if os.path.exists(mix_path) else None
    sym, st = max(by_sym.items(), key=lambda kv: kv[1]['ms'])
    fam, fst = max(by_fam.items(), key=lambda kv: kv[1]['ms'])
    head = kernel_view(sym, st, pmc, sq, mix, False)
    head['share'] = round(st['ms'] / total_ms, 4)
    fv = kernel_view(fam, fst, pmc, sq, mix, True)
    fv['share'] = round(fst['ms'] / total_ms, 4)

    def table(items, k=10):
        top = sorted(items, key=lambda kv: -kv[1]['ms'])[:k]
        return {n: {'share': round(v['ms'] / total_ms, 3), 'avg_us': round(v['ms'] / v['launches'] * 1e3, 1),
                    'launches': v['launches'], 'GBps': round(v['bytes'] / (v['ms'] * 1e-3) / 1e9, 1)} for n, v in top}
    run_bytes = sum(v['bytes'] for v in stats.values())
    # the sort's VALU work (verdict r4 item 3): every kernel's SQ_INSTS_VALU per
    # sort (committed SQ pass of this build, sort only) priced at its mix's
    # measured rate -- the seconds of chip-wide VALU issue the sort needs
    valu_s = None
    if sq and mix:
        valu_s = sum(v['launches'] * v.get('SQ_INSTS_VALU', 0) * 64 * mix[k]['ps_per_lane_instr'] * 1e-12
                     for k, v in sq.items() if k in mix)
    phases = phase_table(phase_rows, total_ms)
    extra = {'phases': phases} if phases else {}
    return {**extra, **head, 'bound': 'hbm', 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'pmc_source': {'traffic': pmc_src, 'sq': sq_src, 'lib_sha256': lib_sha256()},
            'by_symbol': {'kernel': sym, 'note': 'the headline fields above are this kernel'},
            'by_family': fv,
            'clocked_ms_per_sort': round(total_ms, 1),
            'kernels': table(by_sym.items(), 16), 'families': table(by_fam.items(), 8),
            'kernels_by_caller': table(stats.items(), 24),
            # whole sort: every clocked kernel's algorithmic bytes,
            # over its summed kernel time here and over the timed wall in with_run()
            'hbm_achievable_frac': achievable_hbm_frac(),
            'run': {'algorithmic_bytes_per_sort': run_bytes,
                    'GBps_over_kernel_time': round(run_bytes / (total_ms * 1e-3) / 1e9, 1),
                    'valu_s_per_sort': round(valu_s, 5) if valu_s is not None else None}}


def with_run(roof, ms_per_step, world, op_bytes=None):
    """whole-run fractions over the timed wall and world x peak: `run` from the
    kernels' own algorithmic bytes (every kernel launch, including the
    pipeline's intermediate passes), `run_op` from SURVEY §8(d)'s op-level
    formulas (HMult, rotation, ct x pt, ct x const, add, linear sum; each op at
    its level, counted by the engine: Counters::opbytes) summed over ranks"""
    if roof and 'run' in roof:
        gbps = roof['run']['algorithmic_bytes_per_sort'] / (ms_per_step * 1e-3) / 1e9
        roof['run']['GBps_over_wall'] = round(gbps, 1)
        roof['run']['frac_over_wall'] = round(gbps / (world * HBM_PEAK_GBS), 4)
        if roof['run'].get('valu_s_per_sort') is not None:  # one rank's sort over one GPU's VALU
            roof['run']['valu_frac_over_wall'] = round(roof['run']['valu_s_per_sort'] / (ms_per_step * 1e-3), 4)
    if roof is not None and op_bytes:
        gbps = op_bytes / (ms_per_step * 1e-3) / 1e9
        roof['run_op'] = {'op_bytes_per_sort': int(op_bytes), 'GBps_over_wall': round(gbps, 1),
                          'frac_over_wall': round(gbps / (world * HBM_PEAK_GBS), 4)}
    return roof


def cpu_baseline(logN, depth, N, sample_mults, scale_bits, dnum=3):
    """CPU oracle (this repo's C++ restatement, OpenMP) on a bounded sample of
    the same workload: the comparator of one constructRank batch
    (CompositeSign(3,5,2): 35 relinearised products at ring 2^logN, depth 39),
    or `sample_mults` chained relinearised squarings."""
    sys.path.insert(0, os.path.join(REPO, 'oracle'))
    import pyoracle as O
    orc = O.Context(logN, depth, scale_bits, 60, dnum, seed=7)
    rng = np.random.default_rng(1)
    a = orc.encrypt(rng.uniform(0, 1, N), N)
    b = orc.encrypt(rng.uniform(0, 1, N), N)
    cfg = sign_cfg(N)
    orc.reset_counters()
    t = time.perf_counter()
    if sample_mults and sample_mults < 35:
        x = orc.sub(a, b)
        for _ in range(sample_mults):
            x = orc.square(x)
        sample = f'{sample_mults} chained relinearised squarings at ring 2^{logN}, depth {depth}'
    else:
        orc.compare(a, b, *cfg)
        sample = (f'one constructRank comparator batch: Comparison::compare with CompositeSign{cfg} '
                  f'at ring 2^{logN}, depth {depth}')
    dt = time.perf_counter() - t
    c = orc.counters()
    return {'value': round(c['hmult'] / dt, 3), 'unit': 'ciphertext-mults/s', 'cores': O.lib().orc_num_threads(),
            'kind': 'port', 'sample': sample, 'seconds': round(dt, 2), 'hmults': c['hmult']}


def oracle_full_sort(N, logN, depth, scale_bits, ps_split):
    """The CPU oracle's whole sort of this exact configuration, when a golden
    digest recorded one (tests/golden/make_digests.py runs it once, about an
    hour on the build container's CPU; the GPU reproduces its output words,
    tests/test_gpu_digests.py).  Reported beside the bounded sample, never
    re-run here."""
    try:
        with open(os.path.join(REPO, 'tests', 'golden', 'sort_digests.json')) as f:
            digests = json.load(f)
    except (OSError, ValueError):
        return None
    for name, c in digests.items():
        if (c.get('N'), c.get('logN'), c.get('depth'), c.get('scale_bits'), c.get('ps_split', 0)) == \
                (N, logN, depth, scale_bits, 1 if ps_split == 'openfhe' else 0) and 'oracle_sort_s' in c:
            return {'seconds': c['oracle_sort_s'], 'threads': c.get('oracle_threads'), 'digest': name,
                    'where': 'build container (not the GPU box), tests/golden/sort_digests.json',
                    'output': 'word-identical to the GPU sort'}
    return None


def collective_split(ctx, d, dt_rank, steps):
    """rank_compute_ms / allreduce_ms per step, each the max over ranks: the
    engine times every partial-sum exchange from a drained stream to the reduced
    data (fhe_collective_stats), so compute = this rank's wall minus that"""
    st = ctx.collective_stats()
    ar = st['allreduce_s']
    return {'rank_compute_ms': round(d.max(dt_rank - ar) / steps * 1e3, 2),
            'allreduce_ms': round(d.max(ar) / steps * 1e3, 3),
            'allreduce_calls_per_step': round(d.max(float(st['allreduce_calls'])) / steps, 2)}


def make_allreduce(ctx, d):
    """RCCL when every rank has its own GPU, else a host + gloo exchange."""
    if d.world > 1 and d.rccl:
        uid = d.bcast_bytes(F.Context.comm_unique_id() if d.rank == 0 else None)
        ctx.comm_init(uid, d.rank, d.world)
        return None
    if d.world > 1:
        return d.host_allreduce()
    return None


def run_mehp24(a, d):
    """MEHP24 sortLargeArrayFG (src/mehp24/mehp24_sort.cpp:623-645) at the
    reference test's parameters (tests/mehp24/Mehp24SortTest.cpp:26-143: ring
    2^17, scale 2^40, Cfg (3,5,2), dg_i, df_i = 2, parts of 256), N = 4096 by
    default (BASELINE config 5; depth 64 as for 2048).  The P(P+1)/2 pair
    compares and P^2 indicators are sharded over ranks (strong scaling)."""
    N = a.n_sort or 4096
    p = F.mehp24_parameters(N)
    if a.dnum:
        p['dnum'] = a.dnum
    t0 = time.time()
    ctx = F.Context(p['log_ring'], p['depth'] + 1, p['scale_bits'], 60, p['dnum'], seed=a.seed, device=d.device)
    ctx.gen_rotation_keys(p['rots'])
    ctx.set_sort_stack(a.stack)
    allreduce = make_allreduce(ctx, d)
    x = np.random.default_rng(a.seed).permutation(N) / N  # getVectorWithMinDiff(N, 0, 1, 1/N)
    slots = min(N * N, 1 << (p['log_ring'] - 1)) if p['sub'] == 0 else p['sub'] * p['sub']
    ct = ctx.encrypt_ext(x, slots)
    setup_s = time.time() - t0
    shard = (d.rank, d.world)

    def run():
        return ctx.mehp24_sort(ct, N, p['cfg'], p['dg_i'], p['df_i'], p['sub'], shard=shard, allreduce=allreduce)

    out = None
    for _ in range(a.warmup):
        out = run()
    device_sync(ctx)
    d.barrier()
    ctx.reset_counters()
    device_sync(ctx)
    d.barrier()
    prof = ProfRegion(ctx)
    prof.resume()
    t = time.perf_counter()
    for _ in range(a.steps):
        out = run()
    device_sync(ctx)
    d.barrier()
    dt_rank = time.perf_counter() - t
    prof.pause()
    dt = d.max(dt_rank)
    cnt = ctx.counters()
    split = collective_split(ctx, d, dt_rank, a.steps)
    peak_gb = ctx.pool_stats()['peak'] / 1e9
    hm_total = d.sum(cnt['hmult'])
    ks_total = d.sum(cnt['keyswitch'])
    op_total = d.sum(cnt['opbytes'])
    if d.rank == 0:
        y = ctx.decrypt(out)[:N]
        ms = dt / a.steps * 1e3
        P = N // p['sub'] if p['sub'] else 1
        res = {
            'metric': f'MEHP24 encrypted sort seconds + ciphertext-mults/sec, N={N} @ ringDim 2^{p["log_ring"]}',
            'value': round(hm_total / dt, 2),
            'unit': 'ciphertext-mults/s',
            'n_gpus': d.world,
            'steps': a.steps,
            'warmup': a.warmup,
            'ms_per_step': round(ms, 2),
            'sort_seconds': round(ms / 1e3, 4),
            'keyswitches_per_s': round(ks_total / dt, 2),
            'higher_is_better': True,
            'scaling': 'strong',
            'vs_baseline': None,
            'dtype': 'u64',
            'data': 'synthetic: seeded permutation of {k/N}, keys and encryption from a seeded PRNG',
            'config': {'workload': f'MEHP24 sortLargeArrayFG N={N}, parts of {p["sub"]}, ringDim 2^{p["log_ring"]}, '
                                   f'depth {p["depth"]} (+1 FLEXIBLEAUTOEXT), scale 2^{p["scale_bits"]}, dnum '
                                   f'{p["dnum"]}, CompositeSign{p["cfg"]}, indicator ({p["dg_i"]}, {p["df_i"]}), '
                                   f'{len(p["rots"])} rotation keys',
                       'N': N, 'ring_dim': 1 << p['log_ring'], 'mult_depth': p['depth'],
                       'pair_compares': P * (P + 1) // 2, 'indicators': P * P, 'max_stack': a.stack,
                       'parallelism': f'pair/indicator-shard x{d.world}',
                       'collective': {'none': 'none', 'rccl': 'rccl', 'gloo': 'host+gloo (more ranks than GPUs)'}[d.collective]},
            'max_abs_err': float(np.max(np.abs(y - np.sort(x)))),
            'output_level': out.level,
            'hmult_per_sort': int(hm_total / a.steps),
            'setup_s': round(setup_s, 1),
            'hbm_peak_gb_rank0': round(peak_gb, 1),
            **split,
            'roofline': None,
        }
        if not a.no_roofline and d.world == 1:
            try:
                ctx.pool_trim()
                res['roofline'] = with_run(roofline(ctx, run, a.clock_json, 'pmc_traffic_mehp24.json', 'pmc_sq_mehp24.json'),
                                           res['ms_per_step'], 1, op_total / a.steps)
            except Exception as e:  # never hide the main number
                res['roofline'] = {'error': str(e)}
        if not a.no_cpu_baseline:
            try:
                res['cpu_baseline'] = cpu_baseline(p['log_ring'], p['depth'] + 1, N, a.cpu_sample_mults or 6,
                                                   p['scale_bits'], dnum=p['dnum'])
            except Exception as e:
                res['cpu_baseline'] = {'error': str(e)}
        print(json.dumps(res), flush=True)
    d.barrier()


def kway_dg(N):  # d_g of KWaySort235Test (tests/k-way/KWaySort235Test.cpp:97-222)
    return 2 if N <= 16 else 3 if N <= 125 else 4 if N <= 512 else 5


def cpu_bootstrap_baseline(logN, depth, slots, budget):
    """CPU oracle on a bounded sample of the workload: the EvalMod step of one
    bootstrap (Chebyshev degree 88 + 6 double angles: 26 relinearised products
    from level budget_enc down) at the workload's parameters, host cores.  (A
    whole bootstrap would first need ~50 rotation keys generated on the CPU.)"""
    sys.path.insert(0, os.path.join(REPO, 'oracle'))
    import pyoracle as O
    orc = O.Context(logN, depth, 59, 60, 3, seed=7)
    B = O.Bootstrapper(orc, slots, budget, keygen=False)
    x = orc.encrypt(np.random.default_rng(1).uniform(-0.5, 0.5, 2 * slots), 2 * slots, level=budget[0])
    orc.reset_counters()
    t = time.perf_counter()
    B.eval_mod(x)
    dt = time.perf_counter() - t
    c = orc.counters()
    return {'value': round(c['hmult'] / dt, 3), 'unit': 'ciphertext-mults/s', 'cores': O.lib().orc_num_threads(),
            'kind': 'port', 'seconds': round(dt, 2), 'hmults': c['hmult'],
            'sample': f'EvalMod of one bootstrap at ring 2^{logN}, depth {depth}, from level {budget[0]}'}


def run_kway(a, d):
    """kwaySort::Sorter::sorter via KWayAdapter<N>::sort with bootstrapping
    (src/k-way/Sorter.cpp:289-404, EvalUtils.cpp:59-86, src/sign.cpp:164-170)
    in KWaySort235Test's context (tests/k-way/KWaySort235Test.cpp:18-51,
    src/kway_adapter.h:41-63) at ring 2^16 (BASELINE config 4).  Replicas only:
    each rank sorts its own ciphertext."""
    k, M = a.kway_k, a.kway_m
    N = k ** M
    s = 1
    while s < N:
        s *= 2
    budget = (4, 4) if N <= 128 else (5, 5)
    cfg = (3, 2, kway_dg(N))  # CompositeSignConfig(3, d_f, d_g): dg = d_f = 2, df = d_g
    logN, depth = a.log_n, 40
    t0 = time.time()
    ctx = F.Context(logN, depth, 59, 60, 3, seed=a.seed + d.rank, device=d.device)
    B = F.Bootstrapper(ctx, s, budget)
    ctx.gen_rotation_keys(F.kway_rotation_indices(N))
    x = np.random.default_rng(a.seed + d.rank).permutation(N) * (1 - 1e-8) / N  # getVectorWithMinDiff
    ct = ctx.encrypt(x, s)
    setup_s = time.time() - t0

    ctx.set_sort_lanes(a.lanes)  # >= 2: a stage's two comparisons run on two streams

    def run():
        return ctx.kway_sort(ct, k, M, cfg, boot=B)

    out = None
    for _ in range(a.warmup):
        out = run()
    device_sync(ctx)
    d.barrier()
    ctx.reset_counters()
    device_sync(ctx)
    d.barrier()
    prof = ProfRegion(ctx)
    prof.resume()
    t = time.perf_counter()
    for _ in range(a.steps):
        out = run()
    device_sync(ctx)
    d.barrier()
    prof.pause()
    dt = d.max(time.perf_counter() - t)
    cnt = ctx.counters()
    boots = ctx.kway_bootstraps
    peak_gb = ctx.pool_stats()['peak'] / 1e9
    hm_total = d.sum(cnt['hmult'])
    ks_total = d.sum(cnt['keyswitch'])
    op_total = d.sum(cnt['opbytes'])
    y = ctx.decrypt(out)[:N]
    err = d.max(float(np.max(np.abs(y - np.sort(x)))))
    if d.rank == 0:
        ms = dt / a.steps * 1e3
        res = {
            'metric': f'k-way encrypted sort seconds + ciphertext-mults/sec, k={k}, N={N} @ ringDim 2^{logN}',
            'value': round(hm_total / dt, 2),
            'unit': 'ciphertext-mults/s',
            'n_gpus': d.world,
            'steps': a.steps,
            'warmup': a.warmup,
            'ms_per_step': round(ms, 2),
            'sort_seconds': round(ms / 1e3, 4),
            'sorts_per_s': round(d.world * a.steps / dt, 4),
            'keyswitches_per_s': round(ks_total / dt, 2),
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'u64',
            'data': 'synthetic: seeded permutation of {k/N} per rank, keys and encryption from a seeded PRNG',
            'config': {'workload': f'k-way network k={k}, M={M} (N={N}, {s} slots), ringDim 2^{logN}, depth {depth}, '
                                   f'scale 2^59, levelBudget {budget}, CompositeSign{cfg}, bootstrapping',
                       'N': N, 'ring_dim': 1 << logN, 'mult_depth': depth, 'slots': s,
                       'lanes_per_gpu': min(a.lanes, 2), 'parallelism': f'replicas x{d.world}', 'collective': 'none'},
            'max_abs_err': err,
            'output_level': out.level,
            'hmult_per_sort': int(hm_total / a.steps / d.world),
            'checklevel_bootstraps_per_sort': boots,
            'bootstrap_depth': B.depth,
            'setup_s': round(setup_s, 1),
            'hbm_peak_gb_rank0': round(peak_gb, 1),
            'roofline': None,
        }
        if not a.no_roofline:
            try:
                ctx.set_sort_lanes(1)  # the live clock needs one stream
                res['roofline'] = with_run(roofline(ctx, run, a.clock_json, 'pmc_traffic_kway.json', 'pmc_sq_kway.json'),
                                           res['ms_per_step'], 1, op_total / a.steps / d.world)
                ctx.set_sort_lanes(a.lanes)
            except Exception as e:  # never hide the main number
                res['roofline'] = {'error': str(e)}
        if not a.no_cpu_baseline:
            try:
                res['cpu_baseline'] = cpu_bootstrap_baseline(logN, depth, s, budget)
            except Exception as e:
                res['cpu_baseline'] = {'error': str(e)}
        print(json.dumps(res), flush=True)
    d.barrier()


def main():
    a = parse()
    if a.gpus > 1 and not launched_by_torchrun():
        sys.exit(self_launch(a))
    if launched_by_torchrun() and int(os.environ['WORLD_SIZE']) != a.gpus:
        raise SystemExit(f'--gpus {a.gpus} but WORLD_SIZE={os.environ["WORLD_SIZE"]}')
    d = Dist(a.gpus, probe_devices=not a.rendezvous_check)
    if a.rendezvous_check:
        return rendezvous_check(a, d)
    if a.workload == 'mehp24':
        return run_mehp24(a, d)
    if a.workload == 'kway':
        return run_kway(a, d)
    N, logN = a.n_sort or 1024, a.log_n
    depth, rots = F.size_parameters(N)
    cfg = sign_cfg(N)
    t0 = time.time()
    ctx = F.Context(logN, depth, a.scale_bits, 60, 3, seed=a.seed, device=d.device,
                    ps_split=F.PS_SPLIT_OPENFHE if a.ps_split == 'openfhe' else F.PS_SPLIT_ENGINE)
    ctx.gen_rotation_keys(rots)
    ctx.set_sort_lanes(a.lanes)
    ctx.set_sort_stack(a.stack)
    allreduce = make_allreduce(ctx, d)
    x = np.random.default_rng(a.seed).permutation(N) / N  # getVectorWithMinDiff(N, 0, 1, 1/N)
    ct = ctx.encrypt(x, N)
    setup_s = time.time() - t0
    shard = (d.rank, d.world)

    out = None
    cold_s = None
    cold_parts = None
    for i in range(a.warmup):
        if i == 0:  # the first sort encodes every mask (the reference re-encodes them per sort)
            device_sync(ctx)
            d.barrier()
            F.host_stats(reset=True)
            tc = time.perf_counter()
        out = ctx.direct_sort(ct, N, rots, cfg, shard=shard, allreduce=allreduce)
        if i == 0:
            device_sync(ctx)
            cold_parts = F.host_stats(reset=True)
            d.barrier()
            cold_s = d.max(time.perf_counter() - tc)
    device_sync(ctx)
    d.barrier()
    ctx.reset_counters()
    device_sync(ctx)
    d.barrier()
    F.host_stats(reset=True)
    prof = ProfRegion(ctx)
    prof.resume()
    t = time.perf_counter()
    for _ in range(a.steps):
        out = ctx.direct_sort(ct, N, rots, cfg, shard=shard, allreduce=allreduce)
    device_sync(ctx)
    d.barrier()
    dt_rank = time.perf_counter() - t
    prof.pause()
    dt = d.max(dt_rank)
    warm_parts = F.host_stats(reset=True)
    cnt = ctx.counters()
    split = collective_split(ctx, d, dt_rank, a.steps)
    # the reference's per-sort encoding: every mask and checking vector
    # re-encoded (on the device, in batches) at the start of each sort
    masks_ms = None
    if a.mask_steps > 0:
        ctx.set_mask_cache(False)
        device_sync(ctx)
        d.barrier()
        tm = time.perf_counter()
        for _ in range(a.mask_steps):
            ctx.direct_sort(ct, N, rots, cfg, shard=shard, allreduce=allreduce)
        device_sync(ctx)
        d.barrier()
        masks_ms = d.max(time.perf_counter() - tm) / a.mask_steps * 1e3
        mask_parts = F.host_stats(reset=True)
        ctx.set_mask_cache(True)
    peak_gb = ctx.pool_stats()['peak'] / 1e9
    ctx.pool_trim()  # ranks idle at the final barrier hold no cache while rank 0 measures
    d.barrier()
    hm_total = d.sum(cnt['hmult'])
    ks_total = d.sum(cnt['keyswitch'])
    op_total = d.sum(cnt['opbytes'])

    res = None
    if d.rank == 0:
        y = ctx.decrypt(out)
        max_err = float(np.max(np.abs(y - np.sort(x))))
        ms = dt / a.steps * 1e3
        res = {
            'metric': 'encrypted sort seconds + ciphertext-mults/sec, N=1024 @ ringDim 2^16',
            'value': round(hm_total / dt, 2),
            'unit': 'ciphertext-mults/s',
            'n_gpus': d.world,
            'steps': a.steps,
            'warmup': a.warmup,
            'ms_per_step': round(ms, 2),
            'sort_seconds': round(ms / 1e3, 4),
            'keyswitches_per_s': round(ks_total / dt, 2),
            'higher_is_better': True,
            'scaling': 'strong',
            'vs_baseline': None,
            'dtype': 'u64',
            'data': 'synthetic: seeded permutation of {k/N}, keys and encryption from a seeded PRNG',
            'config': {'workload': f'DirectSort N={N}, ringDim 2^{logN}, depth {depth}, scale 2^{a.scale_bits}, '
                                   f'{len(rots)} rotation keys, CompositeSign{cfg}, dnum 3, '
                                   f'{"OpenFHE" if a.ps_split == "openfhe" else "power-of-two"} PS split',
                       'N': N, 'ring_dim': 1 << logN, 'mult_depth': depth, 'scale_bits': a.scale_bits,
                       'ps_split': a.ps_split, 'special_primes': ctx.K, 'lanes_per_gpu': a.lanes,
                       'max_stack': a.stack, 'parallelism': f'batch-shard x{d.world}',
                       'collective': {'none': 'none', 'rccl': 'rccl', 'gloo': 'host+gloo (more ranks than GPUs)'}[d.collective]},
            'max_abs_err': max_err,
            'output_level': out.level,
            'hmult_per_sort': int(hm_total / a.steps),
            'setup_s': round(setup_s, 1),
            # first sort on a fresh context: + every mask/checking-vector encode
            # (src/sort_algo.h:341-342, 714-716 pay these on every sort) and the
            # allocation pool's first growth; null without a warmup step
            'cold_sort_s': round(cold_s, 4) if cold_s is not None else None,
            # rank 0's host costs inside the cold sort (mask / checking-vector
            # encodes -- on the device -- and pool-miss hipMallocs) and inside
            # the timed sorts (none)
            'cold_breakdown': cold_parts,
            'timed_host_costs': warm_parts,
            # wall per sort when every sort re-encodes all its masks on the
            # device first (fhe_set_mask_cache(0)); ms_per_step keeps them cached
            'ms_per_step_masks_per_sort': round(masks_ms, 2) if masks_ms is not None else None,
            'masks_per_sort_breakdown': mask_parts if masks_ms is not None else None,
            'hbm_peak_gb_rank0': round(peak_gb, 1),
            # per sort, max over ranks: a rank's wall outside the partial-sum
            # exchanges, and inside them (header + data all-reduce of both phases)
            **split,
        }
        res['roofline'] = None
        if not a.no_roofline:
            try:
                ctx.set_sort_lanes(1)
                res['roofline'] = with_run(
                    roofline(ctx, lambda: ctx.direct_sort(ct, N, rots, cfg, shard=(0, 1)), a.clock_json),
                    res['ms_per_step'], d.world, op_total / a.steps)
                ctx.set_sort_lanes(a.lanes)
            except Exception as e:  # never hide the main number
                res['roofline'] = {'error': str(e)}
        if not a.no_cpu_baseline:  # rank 0 only, at every world size (the other ranks wait at the barrier)
            try:
                res['cpu_baseline'] = cpu_baseline(logN, depth, N, a.cpu_sample_mults, a.scale_bits)
                full = oracle_full_sort(N, logN, depth, a.scale_bits, a.ps_split)
                if full:
                    res['cpu_baseline']['full_sort'] = full
            except Exception as e:
                res['cpu_baseline'] = {'error': str(e)}
        print(json.dumps(res), flush=True)
    d.barrier()


if __name__ == '__main__':
    main()
