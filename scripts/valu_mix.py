#!/usr/bin/env python3
"""Static VALU instruction mix of every gfx950 kernel (CPU; build container).

Extracts the gfx950 code objects from fhe-sorting_amd/build/device/*.o
(llvm-objcopy + clang-offload-bundler, as tests/test_codeobj.py), disassembles
them and prices each kernel's vector-ALU instructions in full-rate issue slots
with the rates measured on one MI355X (scripts/valu_rates*.hip):
full rate (v_add_u32, v_mov_b32, v_and_b32 ...) 66-69 T lane-ops/s = 1.0;
half rate (v_lshl_add_u64, v_lshrrev_b64, v_mov_b64, v_add3_u32, v_mul_lo_u32,
v_mul_hi_u32 ...) 34-38 T = 1.83; v_mad_u64_u32 23 T = 2.87; a carry or
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
    if re.match(r'v_(add|sub|subrev)(c|b)?_co_', op) or op.startswith('v_cmp') or op.startswith('v_cndmask'):
        return PAIR, 'carry/cmp'
    return 1.0, 'full'


def kernels(obj, tmp):
    fat, co = os.path.join(tmp, 'fat.bin'), os.path.join(tmp, 'gfx950.co')
    subprocess.run([f'{LLVM}/llvm-objcopy', f'--dump-section=.hip_fatbin={fat}', obj, os.devnull], check=True)
    subprocess.run([f'{LLVM}/clang-offload-bundler', '--unbundle', '--type=o', f'--input={fat}',
                    '--targets=hipv4-amdgcn-amd-amdhsa--gfx950', f'--output={co}'], check=True)
    dis = subprocess.run([f'{LLVM}/llvm-objdump', '-d', '--demangle', '--no-show-raw-insn', co], check=True,
                         capture_output=True, text=True).stdout
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
                            'mix': {cl: round(v / n, 3) for cl, v in sorted(classes.items())}}
    json.dump(dict(sorted(table.items())), open(dst, 'w'), indent=1)
    for k, v in sorted(table.items()):
        try:
            print(f"{k:45s} {v['valu_static']:6d} weight {v['weight']:.2f} {v['mix']}")
        except BrokenPipeError:
            break


if __name__ == '__main__':
    main()
