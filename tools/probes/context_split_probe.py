#!/usr/bin/env python3
"""Where a fresh process's HIP context goes: ROCr's ``hsa_init`` (KFD
open, topology, agents) vs HIP's own device set-up (``hipInit``,
``hipSetDevice``, ``hipFree(0)``), over fresh processes in a row
(profiles/r5_boot: the context is 58-100 ms on most boots, 150-270 ms on
some; everything after it is stable).  Torch-free (ROCm 7.2's runtime)
unless ``--torch``.  One JSON line per process.
"""
import argparse
import json
import subprocess
import sys
import time

CHILD = r'''
import ctypes, json, sys, time
torch_first = sys.argv[1] == '1'
t = [time.perf_counter()]
if torch_first:
    import torch  # noqa: F401  (torch's bundled HIP runtime)
    hip = ctypes.CDLL('libamdhip64.so', mode=ctypes.RTLD_GLOBAL)
else:
    hip = ctypes.CDLL('/opt/rocm/lib/libamdhip64.so', mode=ctypes.RTLD_GLOBAL)
hsa = ctypes.CDLL('libhsa-runtime64.so.1', mode=ctypes.RTLD_GLOBAL)
t.append(time.perf_counter())
rc_hsa = hsa.hsa_init()
t.append(time.perf_counter())
if len(sys.argv) > 2 and sys.argv[2] == 'pre':
    # an embryo's shape: ROCr initialised well before HIP is
    time.sleep(1.0)
    slept = time.perf_counter() - t[-1]
    t = [x + slept for x in t]
rc_init = hip.hipInit(0)
t.append(time.perf_counter())
rc_set = hip.hipSetDevice(0)
t.append(time.perf_counter())
rc_free = hip.hipFree(None)
t.append(time.perf_counter())
stream = ctypes.c_void_p()
rc_stream = hip.hipStreamCreate(ctypes.byref(stream))
t.append(time.perf_counter())
names = ('load', 'hsa_init', 'hipInit', 'hipSetDevice', 'hipFree0',
         'stream')
row = {n: round((t[i + 1] - t[i]) * 1e3, 2) for i, n in enumerate(names)}
row['rc'] = [rc_hsa, rc_init, rc_set, rc_free, rc_stream]
print(json.dumps(row))
sys.stdout.flush()
import os
os._exit(0)
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=12)
    ap.add_argument('--torch', action='store_true')
    ap.add_argument('--gap', type=float, default=0.5)
    ap.add_argument('--pre', action='store_true',
                    help='hsa_init, 1 s of sleep, then the HIP calls timed')
    ap.add_argument('--variants', default='',
                    help="comma-separated NAME=VALUE environment variants "
                         "(each its own --n processes; 'default' = as is), "
                         "interleaved process by process")
    args = ap.parse_args()
    import itertools
    import os
    variants = [v for v in args.variants.split(',') if v] or ['default']
    # interleaved, process by process: a slow spell of the box hits every
    # variant alike
    for _, variant in itertools.product(range(args.n), variants):
        env = dict(os.environ)
        if '=' in variant:
            name, _, value = variant.partition('=')
            env[name] = value
        t0 = time.perf_counter()
        out = subprocess.run([sys.executable, '-c', CHILD,
                              '1' if args.torch else '0',
                              'pre' if args.pre else ''],
                             capture_output=True, text=True, timeout=120,
                             env=env)
        line = out.stdout.strip().splitlines()[-1] if out.stdout.strip() \
            else json.dumps({'error': out.stderr[-500:]})
        row = json.loads(line)
        row['process_ms'] = round((time.perf_counter() - t0) * 1e3, 1)
        row['variant'] = variant
        print(json.dumps(row), flush=True)
        time.sleep(args.gap)
    return 0


if __name__ == '__main__':
    sys.exit(main())
