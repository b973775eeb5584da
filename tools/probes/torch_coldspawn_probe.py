#!/usr/bin/env python3
"""Where does a PyTorch worker's cold start go on MI355X?  Stage times of
(a) a fresh process (import torch -> first CUDA call -> weights -> first
forward) and (b) a child forked from a parent that imported torch but never
touched HIP (the zygote design).  One JSON line per variant."""
import json
import os
import sys
import time


def stages(t0, dim=4096, hidden=16384, layers=4, rows=2048):
    out = {}
    import torch
    out['import_torch'] = time.perf_counter() - t0
    torch.zeros(1, device='cuda')
    torch.cuda.synchronize()
    out['cuda_ready'] = time.perf_counter() - t0
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__)))))
    from kiosk_autoscaler_amd.models.torch_engine import TorchMlpEngine

    class Cfg(object):
        pass
    cfg = Cfg()
    cfg.dim, cfg.hidden, cfg.layers, cfg.rows, cfg.batch, cfg.seed = (
        dim, hidden, layers, rows, 1, 7)
    engine = TorchMlpEngine(cfg)
    torch.cuda.synchronize()
    out['weights'] = time.perf_counter() - t0
    engine.warmstart()
    out['warmstart'] = time.perf_counter() - t0
    engine.infer([{'rows': rows, 'seed': 1, 'service_ms': 0}])
    torch.cuda.synchronize()
    out['first_key'] = time.perf_counter() - t0
    return out


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else 'fresh'
    if mode == 'fresh':
        t0 = time.perf_counter()
        print(json.dumps({'mode': 'fresh', 's': stages(t0)}), flush=True)
        return 0
    # zygote: import torch (no HIP), then fork the worker
    t_imp = time.perf_counter()
    import torch  # noqa: F401
    imp = time.perf_counter() - t_imp
    r, w = os.pipe()
    t0 = time.perf_counter()
    pid = os.fork()
    if pid == 0:
        os.close(r)
        out = stages(t0)
        os.write(w, json.dumps(out).encode())
        os._exit(0)
    os.close(w)
    data = b''
    while True:
        chunk = os.read(r, 65536)
        if not chunk:
            break
        data += chunk
    os.waitpid(pid, 0)
    print(json.dumps({'mode': 'zygote', 'parent_import_s': imp,
                      's': json.loads(data)}), flush=True)
    return 0


if __name__ == '__main__':
    sys.exit(main())
