#!/usr/bin/env python3
"""Where does the first RCCL communicator's init time go?

Each configuration runs in a fresh child process (the one-time RCCL init is
per process): load the native module without torch, open the device, then
time each phase of two one-rank communicators (unique id, init, first and
steady 72-byte all-reduce, HBM held, destroy).  One JSON line per
configuration; with ``--debug`` the RCCL INIT log of the default
configuration is kept under ``--out``.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CHILD = r'''
import json, sys, time
sys.path.insert(0, %r)
t0 = time.monotonic()
from kiosk_autoscaler_amd.ops import native
mod = native.load(torch_first=False)
t1 = time.monotonic()
mod.preinit_device(0)
t2 = time.monotonic()
out = {'load_ms': (t1 - t0) * 1e3, 'preinit_ms': (t2 - t1) * 1e3}
free0 = mod.mem_info()[0]
for tag in ('first', 'second'):
    ta = time.monotonic()
    uid = mod.fence_unique_id()
    tb = time.monotonic()
    fence = mod.Fence(uid, 1, 0, 60.0)
    tc = time.monotonic()
    fence.allreduce([1] * 9)
    td = time.monotonic()
    lat = sorted(fence.allreduce([1] * 9)[1] for _ in range(20))
    used = free0 - mod.mem_info()[0]
    te = time.monotonic()
    fence.destroy()
    tf = time.monotonic()
    out.update({tag + '_uid_ms': (tb - ta) * 1e3,
                tag + '_init_ms': (tc - tb) * 1e3,
                tag + '_first_allreduce_ms': (td - tc) * 1e3,
                tag + '_allreduce_us_median': lat[10],
                tag + '_hbm_mb': used / 2.0 ** 20,
                tag + '_destroy_ms': (tf - te) * 1e3})
print(json.dumps(out))
''' % ROOT

CONFIGS = [
    ('default', {}),
    ('env_nchannels_1', {'NCCL_MIN_NCHANNELS': '1', 'NCCL_MAX_NCHANNELS': '1'}),
    ('env_nchannels_1_p2p', {'NCCL_MIN_NCHANNELS': '1',
                             'NCCL_MAX_NCHANNELS': '1',
                             'NCCL_NCHANNELS_PER_NET_PEER': '1',
                             'NCCL_MIN_P2P_NCHANNELS': '1',
                             'NCCL_MAX_P2P_NCHANNELS': '1'}),
    ('no_msccl', {'RCCL_MSCCL_ENABLE': '0', 'RCCL_MSCCLPP_ENABLE': '0'}),
    ('no_ib', {'NCCL_IB_DISABLE': '1'}),
    ('socket_lo', {'NCCL_SOCKET_IFNAME': 'lo', 'NCCL_IB_DISABLE': '1'}),
    ('no_net_plugin', {'NCCL_NET_PLUGIN': 'none', 'NCCL_IB_DISABLE': '1'}),
    ('all', {'RCCL_MSCCL_ENABLE': '0', 'RCCL_MSCCLPP_ENABLE': '0',
             'NCCL_IB_DISABLE': '1', 'NCCL_NET_PLUGIN': 'none',
             'NCCL_SOCKET_IFNAME': 'lo'}),
]


def main():
    parser = argparse.ArgumentParser()
    parser.add_argument('--out', default='gpurun_out/rccl_init')
    parser.add_argument('--debug', action='store_true')
    parser.add_argument('--only', default='')
    args = parser.parse_args()
    os.makedirs(args.out, exist_ok=True)
    configs = list(CONFIGS)
    if args.debug:
        configs.insert(0, ('debug_init', {'NCCL_DEBUG': 'INFO',
                                          'NCCL_DEBUG_SUBSYS': 'INIT,ENV',
                                          'NCCL_DEBUG_FILE': os.path.join(
                                              args.out, 'rccl_init.%h.%p.log')
                                          }))
    for name, extra in configs:
        if args.only and name not in args.only.split(','):
            continue
        env = dict(os.environ, **extra)
        t0 = time.monotonic()
        proc = subprocess.run([sys.executable, '-c', CHILD], env=env,
                              capture_output=True, text=True, timeout=120)
        row = {'config': name, 'env': extra, 'rc': proc.returncode,
               'wall_ms': round((time.monotonic() - t0) * 1e3, 1)}
        lines = proc.stdout.strip().splitlines()
        if proc.returncode == 0 and lines:
            row.update({k: round(v, 1) for k, v in
                        json.loads(lines[-1]).items()})
        else:
            row['stderr'] = proc.stderr[-2000:]
        print(json.dumps(row), flush=True)
        if proc.returncode != 0:
            return proc.returncode
    return 0


if __name__ == '__main__':
    sys.exit(main())
