#!/usr/bin/env python3
"""One worker lifecycle without the autoscaler, for rocprofv3 and timing.

standby preinit (HIP context + code objects) -> Engine (HBM arena, on-device
random init) -> N1 warm-start -> graph capture -> K keys of forward passes.
Prints a JSON line with the host-side stage times; under
``rocprofv3 --kernel-trace --stats`` the per-kernel table shows the
warm-start occupancy (256 WGs) and the N2 GEMM kernels.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    parser = argparse.ArgumentParser()
    parser.add_argument('--dim', type=int, default=4096)
    parser.add_argument('--hidden', type=int, default=16384)
    parser.add_argument('--layers', type=int, default=4)
    parser.add_argument('--rows', type=int, default=2048)
    parser.add_argument('--keys', type=int, default=3)
    parser.add_argument('--passes', type=int, default=20)
    parser.add_argument('--no-preinit', action='store_true')
    parser.add_argument('--with-torch', action='store_true',
                        help='import torch first (round-1 worker)')
    args = parser.parse_args()
    t0 = time.monotonic_ns()
    from kiosk_autoscaler_amd.ops import native
    # like the worker: the native module on ROCm's HIP runtime, no torch
    mod = native.load(torch_first=bool(args.with_torch))
    t_import = time.monotonic_ns()
    pre = {} if args.no_preinit else dict(mod.preinit_device(0))
    t_assign = time.monotonic_ns()
    engine = mod.Engine(0, args.dim, args.hidden, args.layers, args.rows, 1234)
    stages = dict(engine.stage_times())
    warm = dict(engine.warmstart())
    t_warm = time.monotonic_ns()
    engine.prepare(args.rows)
    first = engine.forward(args.rows, 1, 1)
    t_ready = time.monotonic_ns()
    keys = [engine.forward(args.rows, args.passes, k + 2)
            for k in range(args.keys)]
    flops = 2 * 2 * args.rows * args.dim * args.hidden * args.layers
    per_pass = min(k['gpu_ms'] / k['passes'] for k in keys)
    engine.close()
    out = {
        'import_ms': (t_import - t0) / 1e6,
        'preinit_ms': (t_assign - t_import) / 1e6,
        'assign_to_ready_ms': (t_ready - t_assign) / 1e6,
        'engine_stages_ms': {k: round((v - t_assign) / 1e6, 3)
                             for k, v in sorted(stages.items(),
                                                key=lambda kv: kv[1])},
        'warmstart': {k: v for k, v in warm.items() if k != 'cu_mask'},
        'warmstart_done_ms': (t_warm - t_assign) / 1e6,
        'first_forward_gpu_ms': first['gpu_ms'],
        'pass_ms': per_pass,
        'model_tflops': flops / (per_pass * 1e-3) / 1e12,
        'preinit_stages_ms': {k: round((v - t_import) / 1e6, 3)
                              for k, v in pre.items()},
    }
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
