#!/usr/bin/env python3
"""What a deep-idle wake's RCCL generation costs when P fresh processes
load RCCL at once ("at 8 ranks, eight fresh processes
load it at once").

One MI355X cannot hold a multi-rank communicator on one device (RCCL
refuses two ranks per GPU), but the part that grows with the rank count on
a node is each fresh process's one-time load of RCCL's device code (the
``kernels`` phase of its first ``ncclCommInitRank``, ~240 ms of the ~300 ms
of a 1-rank generation).  So P processes open the device, wait at a common
start line, then each builds its first 1-rank communicator at the same
instant, on the one-ISA copy the manager configures
(``parallel/rccl_lib.py``).  Per P: each process's first init and a second
one (warm, what a recycled worker pays).

    python3 tools/probes/rccl_load_contention.py [P ...]   (default 1 2 4 8)

One JSON line per P.  At most 8 children, one at a time per P.
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))


def child():
    sys.path.insert(0, ROOT)
    from kiosk_autoscaler_amd.ops import native
    mod = native.load()
    t0 = time.perf_counter()
    mod.preinit_device(0)
    ctx_ms = (time.perf_counter() - t0) * 1e3
    print('ready', flush=True)
    if sys.stdin.readline().strip() != 'go':
        return
    t0 = time.perf_counter()
    uid = mod.fence_unique_id()
    fence = mod.Fence(uid, 1, 0, 60.0)
    first_ms = (time.perf_counter() - t0) * 1e3
    fence.allreduce([1, 0, 1, 0, 0, 0, 0, 0, 0])
    fence.destroy()
    t0 = time.perf_counter()
    fence = mod.Fence(mod.fence_unique_id(), 1, 0, 60.0)
    warm_ms = (time.perf_counter() - t0) * 1e3
    fence.destroy()
    print(json.dumps({'ctx_ms': round(ctx_ms, 1),
                      'first_init_ms': round(first_ms, 1),
                      'warm_init_ms': round(warm_ms, 1)}), flush=True)


def _line(proc, want):
    """The child's next stdout line starting with ``want`` (RCCL and ROCr
    may print their own lines there first); None at EOF."""
    for line in proc.stdout:
        if line.startswith(want):
            return line
    return None


def _failed(proc):
    try:
        rc = proc.wait(timeout=30)
    except subprocess.TimeoutExpired:
        rc = None
    return RuntimeError('child failed (rc %s): %s' % (
        rc, proc.stderr.read()[-600:]))


def run(p, env):
    procs = [subprocess.Popen([sys.executable, __file__, '--child'], env=env,
                              stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True)
             for _ in range(p)]
    try:
        for proc in procs:
            if _line(proc, 'ready') is None:
                raise _failed(proc)
        t0 = time.perf_counter()
        for proc in procs:
            proc.stdin.write('go\n')
            proc.stdin.flush()
        rows = []
        for proc in procs:
            line = _line(proc, '{')
            if line is None:
                raise _failed(proc)
            rows.append(json.loads(line))
        wall = (time.perf_counter() - t0) * 1e3
        for proc in procs:
            proc.wait(timeout=60)
    finally:
        for proc in procs:
            if proc.poll() is None:
                proc.kill()
                proc.wait()
    first = sorted(r['first_init_ms'] for r in rows)
    warm = sorted(r['warm_init_ms'] for r in rows)
    return {'processes': p, 'wall_ms': round(wall, 1),
            'first_init_ms_mean': round(sum(first) / p, 1),
            'first_init_ms_max': first[-1],
            'warm_init_ms_mean': round(sum(warm) / p, 1),
            'warm_init_ms_max': warm[-1],
            'ctx_ms_max': max(r['ctx_ms'] for r in rows), 'rows': rows}


def main():
    if len(sys.argv) > 1 and sys.argv[1] == '--child':
        child()
        return
    counts = [int(a) for a in sys.argv[1:]] or [1, 2, 4, 8]
    if max(counts) > 8:
        raise SystemExit('at most 8 processes on the device')
    sys.path.insert(0, ROOT)
    from kiosk_autoscaler_amd.parallel import rccl_lib
    env = dict(os.environ)
    info = rccl_lib.configure(env=env)
    print(json.dumps({'rccl_lib': info.get('lib'), 'slim': info.get('slim'),
                      'ms': info.get('ms')}), flush=True)
    for p in counts:
        print(json.dumps(run(p, env)), flush=True)


if __name__ == '__main__':
    main()
