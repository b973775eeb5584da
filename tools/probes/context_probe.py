#!/usr/bin/env python3
"""Does the bench's amdsmi sampler slow a new process's HIP context?

A standby's boot is dominated by its HIP context creation (``hipFree(0)``:
50 ms on most boots, 120-165 ms on some; ``profiles/r4_final3``).  The
bench samples amdsmi (gfx activity, VRAM) every 0.1 s from its own
process.  This probe starts N fresh processes one after another that time
``hipFree(0)`` -- with no sampler, then with the bench's sampler at 10 Hz
and at 2 Hz -- and prints one JSON line per mode (ms: median, max, all).

    python tools/context_probe.py --runs 12
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

CHILD = r'''
import ctypes, time
hip = ctypes.CDLL("libamdhip64.so.7")
t = time.perf_counter()
rc = hip.hipFree(ctypes.c_void_p(0))
print("%.3f %d" % ((time.perf_counter() - t) * 1e3, rc), flush=True)
'''


def run_children(n):
    out = []
    for _ in range(n):
        proc = subprocess.run([sys.executable, '-S', '-c', CHILD],
                              stdout=subprocess.PIPE, timeout=60, check=True,
                              env=dict(os.environ,
                                       LD_LIBRARY_PATH='/opt/rocm/lib'))
        ms, rc = proc.stdout.decode().split()
        if int(rc) != 0:
            raise RuntimeError('hipFree(0) returned %s' % rc)
        out.append(float(ms))
        time.sleep(0.2)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--runs', type=int, default=12)
    args = ap.parse_args()
    from kiosk_autoscaler_amd.bench import gpu_util
    for mode, period in (('none', None), ('amdsmi_10hz', 0.1),
                         ('amdsmi_2hz', 0.5), ('none_again', None)):
        sampler = None
        if period is not None:
            sampler = gpu_util.UtilSampler(period)
            if not sampler.start():
                print(json.dumps({'mode': mode, 'error': sampler.error}))
                continue
        times = run_children(args.runs)
        if sampler is not None:
            sampler.stop()
        times_sorted = sorted(times)
        print(json.dumps({'mode': mode, 'median_ms': times_sorted[
            len(times) // 2], 'max_ms': times_sorted[-1],
            'all_ms': [round(t, 1) for t in times]}), flush=True)
    return 0


if __name__ == '__main__':
    sys.exit(main())
