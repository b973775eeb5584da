#!/usr/bin/env python3
"""L2 fetch of the 4-wave 256x256 GEMM per tile-row group size.

Runs the worker's up-projection (bias + GELU, 2048x16384x4096 by default)
``--reps`` times per ``--group-m`` value, in that order, so that under
``rocprofv3 --pmc FETCH_SIZE ...`` the dispatches split into consecutive
blocks of ``--reps`` per group size:

    rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace --stats \\
        --output-format csv -d gpurun_out/fetch -o f -- \\
        python3 tools/gemm_fetch_probe.py
    python3 tools/gemm_fetch_probe.py --summarize gpurun_out/fetch
"""
import argparse
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))


def summarize(directory, group_ms, reps):
    rows = collections.defaultdict(dict)
    for path in glob.glob(os.path.join(directory, '**',
                                       '*counter_collection*.csv'),
                          recursive=True):
        with open(path) as handle:
            for row in csv.DictReader(handle):
                if 'gemm256_kernel' not in row.get('Kernel_Name', ''):
                    continue
                d = int(row['Dispatch_Id'])
                rows[d][row['Counter_Name']] = \
                    rows[d].get(row['Counter_Name'], 0.0) + \
                    float(row['Counter_Value'])
    ids = sorted(rows)
    out = []
    for i, gm in enumerate(group_ms):
        block = ids[i * reps:(i + 1) * reps][1:]   # first of a block: warm-up
        if not block:
            continue
        mean = {c: sum(rows[d].get(c, 0.0) for d in block) / len(block)
                for c in rows[block[0]]}
        entry = {'group_m': gm, 'dispatches': len(block)}
        if 'FETCH_SIZE' in mean:
            entry['fetch_mb'] = round(mean['FETCH_SIZE'] * 1024 / 1e6, 1)
        for c, v in sorted(mean.items()):
            entry[c] = round(v, 1)
        out.append(entry)
        print(json.dumps(entry))
    return out


def main():
    parser = argparse.ArgumentParser()
    parser.add_argument('--shape', default='2048x16384x4096')
    parser.add_argument('--group-m', default='4,8,2,1')
    parser.add_argument('--reps', type=int, default=6)
    parser.add_argument('--summarize', default='')
    args = parser.parse_args()
    group_ms = [int(g) for g in args.group_m.split(',')]
    if args.summarize:
        summarize(args.summarize, group_ms, args.reps)
        return
    import torch
    from kiosk_autoscaler_amd.ops import kernels, native
    mod = native.load()
    M, N, K = (int(v) for v in args.shape.split('x'))
    a = (torch.rand(M, K, device='cuda') * 2 - 1).to(torch.bfloat16)
    b = ((torch.rand(N, K, device='cuda') * 2 - 1) * 0.05).to(torch.bfloat16)
    bias = torch.randn(N, device='cuda')
    out = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
    ref = None
    default_gm = mod.gemm_group_m()
    try:
        for gm in group_ms:
            mod.gemm_set_group_m(gm)
            for _ in range(args.reps):
                kernels.gemm(a, b, bias=bias, epilogue='gelu', out=out,
                             variant='256w4')
            torch.cuda.synchronize()
            # the tile order must not change the result (bit-identical)
            if ref is None:
                ref = out.clone()
            elif not torch.equal(ref, out):
                raise SystemExit('group_m %d changed the output' % gm)
    finally:
        mod.gemm_set_group_m(default_gm)
    print('ok: %d group sizes, identical outputs' % len(group_ms),
          flush=True)


if __name__ == '__main__':
    main()
