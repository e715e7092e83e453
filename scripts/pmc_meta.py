"""Stamp for the committed PMC tables (profiles/pmc_*.json): the SHA-256 of the
libfhesort.so the counters were collected on.  bench.py reports a table's
traffic / valu_frac only when the stamp equals the loaded library's hash
(bench.py load_table), so counters of one build are never attributed to another.
Environment: FHE_PMC_LIB (default fhe-sorting_amd/lib/libfhesort.so),
FHE_PMC_NOTE (free text: workload, selected region)."""
import hashlib
import os
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def meta():
    lib = os.environ.get('FHE_PMC_LIB') or os.path.join(REPO, 'fhe-sorting_amd', 'lib', 'libfhesort.so')
    h = hashlib.sha256()
    with open(lib, 'rb') as f:
        for chunk in iter(lambda: f.read(1 << 20), b''):
            h.update(chunk)
    return {'lib_sha256': h.hexdigest(), 'collected': time.strftime('%Y-%m-%d %H:%M:%S'),
            'note': os.environ.get('FHE_PMC_NOTE', '')}


def region(rows, name_key='Kernel_Name', id_key='Dispatch_Id'):
    """The rows of a rocprofv3 kernel-trace or counter CSV inside the profiled
    region: dispatches after the last k_region_begin marker and before the
    k_region_end that follows it (bench.py FHE_PROF_REGION=1, one lane so the
    dispatch order is the stream order).  Rows of one dispatch (one per counter)
    stay together.  No markers: every row, and `found` False."""
    ids = {}
    for r in rows:
        ids.setdefault(int(r[id_key]), r[name_key])
    begin = [i for i, n in ids.items() if 'k_region_begin' in n]
    if not begin:
        return rows, False
    b = max(begin)
    ends = [i for i, n in ids.items() if 'k_region_end' in n and i > b]
    e = min(ends) if ends else float('inf')
    return [r for r in rows if b < int(r[id_key]) < e], True
