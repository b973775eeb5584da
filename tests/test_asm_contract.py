"""Static checks of the gfx950 GEMM assembly (CPU: hipcc cross-compiles).

The 4-wave GEMM issues its MFMAs as inline asm (accumulators pinned to
AGPRs), for which hipcc inserts no wait states: the kernels must not spill
and must not touch an accumulator before the drain that ends the k-loop.
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not shutil.which(os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')),
                    reason='hipcc not available')
def test_four_wave_gemm_asm_contract():
    proc = subprocess.run([sys.executable,
                           os.path.join(ROOT, 'tools', 'check_asm_mfma.py')],
                          stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                          text=True, timeout=600)
    assert proc.returncode == 0, proc.stdout[-3000:]
    # 9 gemm256_kernel<., 256, 4, .> instantiations (the spilling persistent
    # bias+GELU one is gone, round 6) + 4 gemm256p_kernel
    assert 'checked 13 4-wave kernels: ok' in proc.stdout


def test_checker_flags_violations():
    sys.path.insert(0, os.path.join(ROOT, 'tools'))
    import check_asm_mfma
    name = '_ZN5kiosk12_GLOBAL__N_114gemm256_kernelILi0ELi256ELi4EEEvPKt'
    good = '\n'.join([name + ':', '\tv_mfma_f32_16x16x32_bf16 a[0:3], v[0:3], '
                      'v[4:7], a[0:3]', '\ts_waitcnt vmcnt(0)', '\ts_nop 7',
                      '\tv_accvgpr_read_b32 v8, a0', '.Lfunc_end0:'])
    assert check_asm_mfma.check(good)[1] == []
    bad = good.replace('\ts_waitcnt vmcnt(0)',
                       '\tv_accvgpr_read_b32 v9, a1')
    assert check_asm_mfma.check(bad)[1]
    spill = good.replace('\ts_waitcnt vmcnt(0)',
                         '\tscratch_store_dword off, v1, off')
    assert check_asm_mfma.check(spill)[1]
