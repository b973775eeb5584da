#!/usr/bin/env python3
"""Where a fresh worker process's device open goes (``preinit_device``).

Each configuration runs in its own fresh interpreter (a cold HIP runtime,
as a zygote-forked worker has), ``--reps`` times:

* ``preinit``: ``preinit_device(0)`` alone -- what a cold spawn pays:
  context, kernel attributes, every kernel's first launch, one sync;
* ``split``: ``preload_modules(0)`` (context + kernel attributes) first,
  then ``preinit_device(0)``: the second call's time is the launches (first
  launch of every GEMM variant, scratch allocation, stream, one sync).

    python3 tools/preinit_probe.py --reps 5 > gpurun_out/preinit.jsonl
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
sys.path.insert(0, %(root)r)
t0 = time.monotonic_ns()
from kiosk_autoscaler_amd.ops import native
mod = native.load()
t1 = time.monotonic_ns()
out = {'import_ms': (t1 - t0) / 1e6}
if %(split)r:
    pre = dict(mod.preload_modules(0))
    out['preload_context_ms'] = (pre['preload_context'] - pre['preload_enter']) / 1e6
    out['preload_prepare_ms'] = (pre['preload_done'] - pre['preload_context']) / 1e6
st = dict(mod.preinit_device(0))
out['preinit_context_ms'] = (st['preinit_context'] - st['preinit_enter']) / 1e6
out['preinit_launches_ms'] = (st['preinit_done'] - st['preinit_context']) / 1e6
out['preinit_total_ms'] = (st['preinit_done'] - st['preinit_enter']) / 1e6
print(json.dumps(out))
'''


def main():
    parser = argparse.ArgumentParser()
    parser.add_argument('--reps', type=int, default=5)
    args = parser.parse_args()
    for config in ('preinit', 'split'):
        for rep in range(args.reps):
            code = CHILD % {'root': ROOT, 'split': config == 'split'}
            t0 = time.monotonic()
            proc = subprocess.run([sys.executable, '-S', '-c', code],
                                  capture_output=True, text=True, timeout=120)
            wall = (time.monotonic() - t0) * 1e3
            if proc.returncode != 0:
                sys.stderr.write(proc.stderr)
                return proc.returncode
            line = json.loads(proc.stdout.strip().splitlines()[-1])
            line.update(config=config, rep=rep, process_wall_ms=round(wall, 1))
            print(json.dumps(line), flush=True)
    return 0


if __name__ == '__main__':
    sys.exit(main())
