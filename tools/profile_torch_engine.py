#!/usr/bin/env python3
"""The PyTorch-ROCm engine's lifecycle for rocprofv3: a standby's boot
(``preinit_device``, ``warm_device``), the engine build (one DLPack arena,
weights by the init kernel, forward + warm-start native hipGraphs), READY (one
warm-start graph launch) and K keys of forward passes.

Under ``rocprofv3 --kernel-trace --stats`` the kernel table shows that the
work a torch process runs is ours: the gemm256 GEMMs with fused epilogues,
the split-K reduce, the partial sums and the 256-workgroup warm start.
Prints one JSON line with host-side timings.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--model', default='4096x16384x4')
    ap.add_argument('--rows', type=int, default=2048)
    ap.add_argument('--keys', type=int, default=3)
    ap.add_argument('--passes', type=int, default=20)
    args = ap.parse_args()
    import torch
    from kiosk_autoscaler_amd.ops import native
    from kiosk_autoscaler_amd.models.torch_kiosk import TorchKioskEngine
    from kiosk_autoscaler_amd.worker.runtime import WorkerConfig
    mod = native.load()
    out = {}
    t0 = time.perf_counter()
    mod.preinit_device(0)
    TorchKioskEngine.warm_device()
    out['boot_ms'] = (time.perf_counter() - t0) * 1e3
    cfg = WorkerConfig({'MODEL': args.model, 'ROWS_PER_KEY': str(args.rows)},
                       {'worker_id': 'profile'})
    t0 = time.perf_counter()
    engine = TorchKioskEngine(cfg)
    out['build_ms'] = (time.perf_counter() - t0) * 1e3
    engine.warmstart()                      # first run of the graph
    t0 = time.perf_counter()
    info = engine.warmstart()
    out['ready_ms'] = (time.perf_counter() - t0) * 1e3
    out['warm_blocks'] = info['blocks']
    walls = []
    for key in range(args.keys):
        t0 = time.perf_counter()
        for _ in range(args.passes):
            engine.forward(args.rows, key)
        engine.stream.synchronize()
        walls.append((time.perf_counter() - t0) * 1e3 / args.passes)
        out.setdefault('checksums', []).append(engine.checksum())
    out['forward_ms'] = walls
    dim, hidden, layers = cfg.dim, cfg.hidden, cfg.layers
    flops = 2.0 * args.rows * dim * hidden * 2 * layers
    out['forward_pflops'] = flops / (min(walls) / 1e3) / 1e15
    engine.close()
    torch.cuda.synchronize()
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    sys.exit(main())
