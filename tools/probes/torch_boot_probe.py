#!/usr/bin/env python3
"""Where does a PyTorch standby's boot go, next to the torch-free one's?

Each row is a fresh child process (the parent never touches the GPU) that
does what a woken standby does: import (torch first for ``--torch``), open
the device (``preinit_device``: context, launch handles, one run of every
kernel), the plug-in's ``warm_device`` hook, then the engine build and the
first warm start.  Stage times in ms from the child's start; the engine
build's own stages (``TorchKioskEngine``'s ``stage`` callback) are relative
to the build's start.  One JSON line per child.

    python tools/torch_boot_probe.py --repeat 3
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child(use_torch, model):
    t_start = time.perf_counter()
    row = {'torch': use_torch,
           'torch_stream_first': bool(os.environ.get(
               'PROBE_TORCH_STREAM_FIRST'))}

    def mark(name):
        row[name] = round((time.perf_counter() - t_start) * 1e3, 2)
    sys.path.insert(0, ROOT)
    from kiosk_autoscaler_amd.ops import native
    # the worker's order: native.load imports torch (after mapping ROCm's
    # comgr, ``prefer_rocm_comgr``), then the extension
    mod = native.load(torch_first=use_torch)
    mark('native_loaded')
    with open('/proc/self/maps') as maps:
        row['comgr'] = sorted({line.split()[-1] for line in maps
                               if 'comgr' in line})
    if use_torch and os.environ.get('PROBE_TORCH_STREAM_FIRST'):
        # which pays the first hardware queue: torch's own stream, created
        # before preinit_device creates the native one?
        import torch
        torch.cuda.init()
        mark('torch_cuda_init')
        torch.empty(1, device='cuda').zero_()
        torch.cuda.synchronize()
        mark('torch_null_stream_op')
        side = torch.cuda.Stream()
        with torch.cuda.stream(side):
            torch.empty(1, device='cuda').zero_()
        side.synchronize()
        mark('torch_side_stream_op')
    stages = dict(mod.preinit_device(0))
    base = stages['preinit_enter']
    row['preinit'] = {k: round((v - base) / 1e6, 2) for k, v in stages.items()}
    mark('preinit_done')
    dim, hidden, layers = (int(x) for x in model.split('x'))
    if use_torch:
        from kiosk_autoscaler_amd.models.torch_kiosk import TorchKioskEngine
        from kiosk_autoscaler_amd.worker.runtime import WorkerConfig
        TorchKioskEngine.warm_device()
        mark('warm_device_done')
        cfg = WorkerConfig({'MODEL_DIM': str(dim), 'MODEL_HIDDEN': str(hidden),
                            'MODEL_LAYERS': str(layers),
                            'ROWS_PER_KEY': '2048'}, {'worker_id': 'probe'})
        build = {}
        t0 = time.perf_counter()

        def stage(name, t=None):
            build[name] = round((time.perf_counter() - t0) * 1e3, 2)
        engine = TorchKioskEngine(cfg, stage)
        row['build'] = build
    else:
        engine = mod.Engine(0, dim, hidden, layers, 2048, 1)
    mark('engine_built')
    engine.warmstart()
    mark('first_warmstart')
    t0 = time.perf_counter()
    engine.warmstart()
    row['ready_ms'] = round((time.perf_counter() - t0) * 1e3, 3)
    if use_torch:
        import torch
        a = torch.randn(512, 512, device='cuda', dtype=torch.bfloat16)
        row['torch_matmul_ok'] = bool(torch.isfinite((a @ a).float()).all())
        with open('/proc/self/maps') as maps:
            row['hip_runtime'] = sorted({line.split()[-1] for line in maps
                                         if 'libamdhip64' in line})
    engine.close()
    print(json.dumps(row), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--child', choices=('torch', 'native'))
    ap.add_argument('--repeat', type=int, default=3)
    ap.add_argument('--model', default='4096x16384x4')
    args = ap.parse_args()
    if args.child:
        child(args.child == 'torch', args.model)
        return 0
    for _ in range(args.repeat):
        for kind, first in (('native', ''), ('torch', ''), ('torch', '1')):
            env = dict(os.environ, PROBE_TORCH_STREAM_FIRST=first)
            out = subprocess.run(
                [sys.executable, os.path.abspath(__file__), '--child', kind,
                 '--model', args.model], env=env,
                stdout=subprocess.PIPE, timeout=300, check=True)
            sys.stdout.write(out.stdout.decode())
            sys.stdout.flush()
    return 0


if __name__ == '__main__':
    sys.exit(main())
