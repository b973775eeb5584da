#!/usr/bin/env python3
"""Static check of the 4-wave GEMM kernels' asm-MFMA contract.

hipcc pads no wait states after an inline-asm MFMA (cdna_hip_programming.md
§5.7), so in every ``gemm256_kernel<*, 256, 4, *>`` and ``gemm256p_kernel<*>``
the accumulators (AGPRs)
may be touched only by MFMAs until the ``s_nop`` drain that ends the k-loop,
and no scratch (spill) access may appear anywhere -- except, in the
persistent variant (``kPersist`` = 1: a loop over tiles around it all), a
spill outside the k-loop (a reload or two per tile, never per MFMA).  This
script compiles csrc/kernels/gemm256.hip to gfx950 assembly and fails if
either rule is broken.

    python tools/check_asm_mfma.py
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
AGPR = re.compile(r'\ba(\d+|\[\d+:\d+\])')


def check(asm_text):
    problems = []
    # the 4-wave kernels and the two-waves-per-SIMD arm (gemm256p_kernel):
    # both issue their MFMAs as AGPR-pinned inline asm
    funcs = re.findall(r'^(_Z\S*(?:gemm256_kernelILi\dELi256ELi4E|'
                       r'gemm256p_kernelILi\d)\S*):', asm_text, re.M)
    if not funcs:
        problems.append('no 4-wave gemm256 kernel found')
    for name in funcs:
        start = asm_text.index(name + ':')
        end = asm_text.index('.Lfunc_end', start)
        body = [l.strip() for l in asm_text[start:end].split('\n')]
        insts = [l for l in body if l and not l.startswith(('.', ';'))]
        persistent = re.search(r'ELi256ELi4ELi\dELi1EE', name) is not None
        scratch = [i for i, l in enumerate(insts) if l.startswith('scratch_')]
        # last MFMA before the drain: everything between must not touch AGPRs
        drain = [i for i, l in enumerate(insts) if l.startswith('s_nop 7')]
        if not drain:
            problems.append('%s: no s_nop drain' % name)
            continue
        first_drain = drain[0]
        last_mfma = max((i for i, l in enumerate(insts[:first_drain])
                         if l.startswith('v_mfma')), default=None)
        if last_mfma is None:
            problems.append('%s: no MFMA before the drain' % name)
            continue
        first_mfma = min(i for i, l in enumerate(insts)
                         if l.startswith('v_mfma'))
        hot = [i for i in scratch if first_mfma <= i <= last_mfma]
        if hot or (scratch and not persistent):
            problems.append('%s: scratch (spill) access%s' % (
                name, ' in the k-loop' if hot else ''))
        for l in insts[last_mfma + 1:first_drain]:
            if AGPR.search(l.split(';')[0]) and not l.startswith('v_mfma'):
                problems.append('%s: AGPR touched before the drain: %s'
                                % (name, l))
    return funcs, problems


def main():
    with tempfile.TemporaryDirectory() as tmp:
        out = os.path.join(tmp, 'gemm256.s')
        subprocess.check_call([
            HIPCC, '-O3', '-std=c++17', '--offload-arch=gfx950',
            '--cuda-device-only', '-S', '-I', os.path.join(ROOT, 'csrc',
                                                         'kernels'),
            os.path.join(ROOT, 'csrc', 'kernels', 'gemm256.hip'), '-o', out])
        text = open(out).read()
    funcs, problems = check(text)
    for p in problems:
        print('FAIL', p)
    print('checked %d 4-wave kernels: %s' % (
        len(funcs), 'ok' if not problems else '%d problem(s)' % len(problems)))
    return 1 if problems else 0


if __name__ == '__main__':
    sys.exit(main())
