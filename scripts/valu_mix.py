#!/usr/bin/env python3
"""Static VALU instruction mix of every gfx950 kernel (CPU; build container).

Extracts the gfx950 code objects from fhe-sorting_amd/build/device/*.o
(llvm-objcopy + clang-offload-bundler, as tests/test_codeobj.py), disassembles
them and prices each kernel's vector-ALU instructions in full-rate issue slots
with the rates measured on one MI355X (scripts/valu_rates*.hip):
full rate (v_add_u32, v_mov_b32, v_and_b32 ...) 66-69 T lane-ops/s = 1.0;
half rate (v_lshl_add_u64, v_lshrrev_b64, v_mov_b64, v_add3_u32, v_mul_lo_u32,
v_mul_hi_u32 ...) 34-38 T = 1.83, and the fp64 forms (v_fma_f64, v_mul_f64,
v_add_f64, v_rndne_f64, v_floor_f64, v_cvt_*_f64: 33-38 T, round 5's
valu_rates3.hip, profiles/r5_rates) at the same half rate; v_mad_u64_u32 23 T = 2.87; a carry or
compare/select pair (v_add_co + v_addc_co, v_cmp + v_cndmask) 19-20 T pairs =
1.69 per instruction.  `weight` = average slots per VALU instruction of the
kernel's code (static: unrolled bodies dominate these kernels), and
ps_per_lane_instr = weight / 67.5 T: bench.py's roofline.valu_frac is
SQ_INSTS_VALU x 64 lanes x ps_per_lane_instr / launch duration -- the share of
the measured VALU throughput the launch used.
usage: valu_mix.py [out.json]   (default profiles/valu_mix.json)
"""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(REPO, 'fhe-sorting_amd', 'build', 'device')
LLVM = '/opt/rocm/lib/llvm/bin'

FULL_T = 67.5  # measured lane-instructions per second, x 1e12
MAD = FULL_T / 23.0
HALF = FULL_T / 36.0
PAIR = FULL_T / 39.0
HALF_OPS = {'v_lshl_add_u64', 'v_lshlrev_b64', 'v_lshrrev_b64', 'v_ashrrev_i64', 'v_mov_b64', 'v_add3_u32',
            'v_mul_lo_u32', 'v_mul_hi_u32', 'v_mul_hi_i32', 'v_lshl_or_b32', 'v_add_u64', 'v_sub_u64'}


def cost(op):
    if op.startswith('v_mad_u64_u32') or op.startswith('v_mad_i64_i32'):
        return MAD, 'mad64'
    if op in HALF_OPS:
        return HALF, 'half'
    if op.endswith('_f64') or '_f64_' in op:
        return HALF, 'f64'
    if re.match(r'v_(add|sub|subrev)(c|b)?_co_', op) or op.startswith('v_cmp') or op.startswith('v_cndmask'):
        return PAIR, 'carry/cmp'
    return 1.0, 'full'


def occupancy(co):
    """waves per SIMD of every kernel of a code object from its metadata notes:
    the unified 512-entry VGPR file (VGPR + AGPR, granule 8) and the 160-KiB LDS
    per CU over blocks of max_flat_workgroup_size threads, at most 8"""
    notes = subprocess.run([f'{LLVM}/llvm-readelf', '--notes', co], check=True, capture_output=True, text=True).stdout
    out, cur = {}, {}

    def flush():
        if '.name' not in cur:
            return
        dem = subprocess.run(['c++filt', cur['.name']], capture_output=True, text=True).stdout.strip()
        k = re.search(r'(k_[a-z0-9_]+(<[^()]*?>)?)\(', dem)
        if not k:
            return
        regs = cur.get('.vgpr_count', 0) + cur.get('.agpr_count', 0)
        alloc = max(8, -(-regs // 8) * 8)
        w = min(8, 512 // alloc)
        lds, wg = cur.get('.group_segment_fixed_size', 0), cur.get('.max_flat_workgroup_size', 256)
        if lds:
            w = min(w, (160 * 1024 // lds) * max(1, wg // 64) // 4)
        out[k.group(1).replace('(anonymous namespace)::', '')] = {'waves_per_simd': w, 'vgprs': regs, 'lds': lds}

    for line in notes.splitlines():
        m = re.match(r'^\s+(-\s+)?(\.[a-z_]+):\s+(\S+)\s*$', line)
        if not m:
            continue
        if m.group(1):  # a new kernel entry
            flush()
            cur = {}
        key, val = m.group(2), m.group(3)
        cur[key] = int(val) if val.isdigit() else val
    flush()
    return out


def kernels(obj, tmp):
    fat, co = os.path.join(tmp, 'fat.bin'), os.path.join(tmp, 'gfx950.co')
    subprocess.run([f'{LLVM}/llvm-objcopy', f'--dump-section=.hip_fatbin={fat}', obj, os.devnull], check=True)
    subprocess.run([f'{LLVM}/clang-offload-bundler', '--unbundle', '--type=o', f'--input={fat}',
                    '--targets=hipv4-amdgcn-amd-amdhsa--gfx950', f'--output={co}'], check=True)
    dis = subprocess.run([f'{LLVM}/llvm-objdump', '-d', '--demangle', '--no-show-raw-insn', co], check=True,
                         capture_output=True, text=True).stdout
    kernels.occ.update(occupancy(co))
    out, name = {}, None
    for line in dis.splitlines():
        m = re.match(r'^[0-9a-f]+ <(.*)>:$', line)
        if m:
            full = m.group(1)
            k = re.search(r'(k_[a-z0-9_]+(<[^()]*?>)?)\(', full)
            name = k.group(1).replace('(anonymous namespace)::', '') if k else None
            if name and name not in out:
                out[name] = collections.Counter()
            continue
        if not name:
            continue
        m = re.match(r'^\s+(v_[a-z0-9_]+)', line)
        if m and not m.group(1).startswith('v_mfma'):
            out[name][m.group(1)] += 1
    return out


kernels.occ = {}


def main():
    dst = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, 'profiles', 'valu_mix.json')
    table = {}
    with tempfile.TemporaryDirectory() as tmp:
        for obj in ('ntt.o', 'kernels.o'):
            for k, c in kernels(os.path.join(BUILD, obj), tmp).items():
                n = sum(c.values())
                if not n:
                    continue
                classes = collections.Counter()
                slots = 0.0
                for op, cnt in c.items():
                    w, cls = cost(op)
                    slots += w * cnt
                    classes[cls] += cnt
                # seconds of chip-wide VALU issue per lane-instruction of this mix
                # (weight / 67.5e12): valu_frac = SQ_INSTS_VALU * 64 * s / duration
                table[k] = {'valu_static': n, 'weight': round(slots / n, 3),
                            'ps_per_lane_instr': round(slots / n / FULL_T, 6),
                            'mix': {cl: round(v / n, 3) for cl, v in sorted(classes.items())},
                            **kernels.occ.get(k, {})}
    json.dump(dict(sorted(table.items())), open(dst, 'w'), indent=1)
    for k, v in sorted(table.items()):
        try:
            print(f"{k:45s} {v['valu_static']:6d} weight {v['weight']:.2f} {v['mix']}")
        except BrokenPipeError:
            break


if __name__ == '__main__':
    main()
