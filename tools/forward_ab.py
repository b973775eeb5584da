#!/usr/bin/env python3
"""A/B of the worker forward under the split-K combine modes (interleaved
rounds in one process, cdna_hip_programming.md §5.4 rule 24): prints one
JSON line with the per-mode forward times (median / min over rounds) and
checks every mode's output elementwise against the fp32 reference."""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    parser = argparse.ArgumentParser()
    parser.add_argument('--rows', type=int, default=2048)
    parser.add_argument('--dim', type=int, default=4096)
    parser.add_argument('--hidden', type=int, default=16384)
    parser.add_argument('--layers', type=int, default=4)
    parser.add_argument('--modes', default='0,1')
    parser.add_argument('--rounds', type=int, default=9)
    parser.add_argument('--passes', type=int, default=20)
    args = parser.parse_args()
    import torch
    from kiosk_autoscaler_amd.ops import kernels, native
    mod = native.load()
    modes = [int(m) for m in args.modes.split(',')]
    default = mod.gemm_splitk_fused()
    engines = {}
    check = {}
    try:
        for mode in modes:
            # the mode is read at graph capture: one engine per mode
            mod.gemm_set_splitk_fused(mode)
            eng = mod.Engine(0, args.dim, args.hidden, args.layers, args.rows,
                             5)
            out, ref, stats = kernels.compare_engine_forward(eng, args.rows,
                                                             5, 9)
            torch.testing.assert_close(out, ref, rtol=3e-2, atol=3e-2)
            check[mode] = stats['max_abs_err']
            engines[mode] = eng
        mod.gemm_set_splitk_fused(default)
        times = {m: [] for m in modes}
        for _ in range(args.rounds):
            for mode, eng in engines.items():
                r = eng.forward(args.rows, args.passes, 1)
                times[mode].append(r['gpu_ms'] / args.passes)
    finally:
        for eng in engines.values():
            eng.close()
        mod.gemm_set_splitk_fused(default)
    flops = args.layers * 2 * 2.0 * args.rows * args.dim * args.hidden
    print(json.dumps({
        'shape': [args.rows, args.dim, args.hidden, args.layers],
        'forward_ms': {str(m): {'median': statistics.median(t),
                                'min': min(t)} for m, t in times.items()},
        'pflops_median': {str(m): flops / (statistics.median(t) * 1e-3)
                          / 1e15 for m, t in times.items()},
        'max_abs_err': {str(m): e for m, e in check.items()}}))


if __name__ == '__main__':
    main()
