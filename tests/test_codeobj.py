"""Build guard on the gfx950 code objects (CPU): no hot kernel spills registers
to scratch.  A spill slipped in once this round -- the lazy forward reduction
schedule made the compiler spill the ring-2^17 column pass (132 VGPRs + 272 B
of scratch, 3.3x slower, MEHP24 14.95 -> 21.6 s) with every result still
correct -- so the kernel metadata of the built objects is checked here:
`.private_segment_fixed_size` must be 0 for every kernel except the 512-point
row passes, which only rings >= 2^18 would launch (no configuration does)."""
import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(REPO, 'fhe-sorting_amd', 'build', 'device')
LLVM = '/opt/rocm/lib/llvm/bin'
ALLOW = re.compile(r'k_ntt_fwdILi9ELi5ELb0E')  # k_ntt_fwd<9, 5, false, ...>: ring >= 2^18 rows


def _kernels(obj, tmp):
    fat, co = os.path.join(tmp, 'fat.bin'), os.path.join(tmp, 'gfx950.co')
    subprocess.run([f'{LLVM}/llvm-objcopy', f'--dump-section=.hip_fatbin={fat}', obj, os.devnull], check=True)
    subprocess.run([f'{LLVM}/clang-offload-bundler', '--unbundle', '--type=o', f'--input={fat}',
                    '--targets=hipv4-amdgcn-amd-amdhsa--gfx950', f'--output={co}'], check=True)
    notes = subprocess.run([f'{LLVM}/llvm-readelf', '--notes', co], check=True, capture_output=True,
                           text=True).stdout
    out, name = {}, None
    for line in notes.splitlines():
        m = re.search(r'\.name:\s+(\S+)', line)
        if m:
            name = m.group(1)
        m = re.search(r'\.private_segment_fixed_size:\s+(\d+)', line)
        if m and name:
            out[name] = int(m.group(1))
    return out


@pytest.mark.skipif(not os.path.exists(f'{LLVM}/clang-offload-bundler'), reason='ROCm LLVM tools missing')
@pytest.mark.parametrize('obj', ['ntt.o', 'kernels.o'])
def test_no_scratch_spills(obj, tmp_path):
    path = os.path.join(BUILD, obj)
    assert os.path.exists(path), f'{path} not built (run __graft_entry__.build())'
    k = _kernels(path, str(tmp_path))
    assert len(k) > 10, 'no kernel metadata found'
    spills = {n: b for n, b in k.items() if b and not ALLOW.search(n)}
    assert not spills, f'kernels spilling to scratch: {spills}'
