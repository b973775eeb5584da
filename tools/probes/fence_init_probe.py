#!/usr/bin/env python3
"""Time RCCL communicator set-up for the N4 fence (world size 1) under
environment variants, each in a fresh child process (env must be set
before RCCL loads).  Prints one JSON line per variant:
{variant, warmup_ms, inits_ms[...], allreduce_us}."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

VARIANTS = {
    'default': {},
    'no_msccl': {'RCCL_MSCCL_ENABLE': '0', 'RCCL_MSCCLPP_ENABLE': '0'},
    'no_net': {'NCCL_IB_DISABLE': '1', 'NCCL_NET_PLUGIN': 'none'},
    'proto_simple': {'NCCL_PROTO': 'Simple', 'NCCL_ALGO': 'Ring'},
    'one_channel': {'NCCL_MIN_NCHANNELS': '1', 'NCCL_MAX_NCHANNELS': '1'},
    'lazy_connect': {'NCCL_RUNTIME_CONNECT': '1'},
    'all': {'RCCL_MSCCL_ENABLE': '0', 'RCCL_MSCCLPP_ENABLE': '0',
            'NCCL_IB_DISABLE': '1', 'NCCL_NET_PLUGIN': 'none',
            'NCCL_MIN_NCHANNELS': '1', 'NCCL_MAX_NCHANNELS': '1',
            'NCCL_RUNTIME_CONNECT': '1'},
}


def child():
    sys.path.insert(0, ROOT)
    import torch  # noqa: F401
    from kiosk_autoscaler_amd.ops import native
    mod = native.load()
    mod.preinit_device(0)
    t0 = time.perf_counter()
    mod.fence_warmup(60.0)
    warm = (time.perf_counter() - t0) * 1e3
    inits = []
    us = None
    for _ in range(3):
        uid = mod.fence_unique_id()
        t0 = time.perf_counter()
        fence = mod.Fence(uid, 1, 0, 60.0)
        inits.append(round((time.perf_counter() - t0) * 1e3, 1))
        _, us = fence.allreduce([1, 0, 1, 0, 0, 0, 0, 0, 0])
        fence.destroy()
    print(json.dumps({'warmup_ms': round(warm, 1), 'inits_ms': inits,
                      'allreduce_us': round(us, 1)}))


def main():
    if len(sys.argv) > 1 and sys.argv[1] == '--child':
        child()
        return
    names = sys.argv[1:] or list(VARIANTS)
    for name in names:
        env = dict(os.environ, **VARIANTS[name])
        proc = subprocess.run([sys.executable, __file__, '--child'], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True, timeout=240)
        line = proc.stdout.strip().splitlines()[-1] if proc.stdout.strip() \
            else '{}'
        out = json.loads(line) if line.startswith('{') else {}
        out['variant'] = name
        out['rc'] = proc.returncode
        if proc.returncode:
            out['err'] = proc.stderr[-400:]
        print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
