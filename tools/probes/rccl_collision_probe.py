#!/usr/bin/env python3
"""Root cause of VERDICT r3 missing-1: what does a serving (or starting)
worker wait on while an RCCL generation initialises in its process?

Each mode runs in a fresh child process (RCCL's one-time costs are per
process).  The child opens the device, builds the production engine
(4 x 4096->16384->4096, 2048 rows, hipGraph forward) and then, while a
*collider* runs the node communicator's first generation (``ncclGetUniqueId``
-> ``ncclCommInitRank`` (1 rank) -> 72-B all-reduce -> destroy), the main
thread keeps doing worker work and timestamps every call:

* ``forward``: graph launches of the forward (what a serving worker does);
* ``build``: a fresh Engine (weights, arena, graph capture) + warm-start
  kernel per iteration (what an assignment on a fresh standby does);
* ``ready``: the warm-start alone on a built engine (what an assignment on
  a standby with a prebuilt engine does before READY).

Collider placement:

* ``inproc``   -- a thread of the same process (today's node agent);
* ``sidecar``  -- a separate process pinned to the same GPU;
* ``none``     -- no collider (the baseline distribution).

One JSON line per (mode, work): the collider's phase intervals (monotonic
ns) and, for the worker calls that overlapped each phase, count / median /
max wall ms, against the no-collider median.  Run it under
``rocprofv3 --hip-trace --kernel-trace`` to see which HIP API call of the
worker thread carries the wait.
"""
import argparse
import json
import os
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

PHASES = ('uid', 'init', 'allreduce', 'destroy')


def sample_syscalls(tid, out, stop):
    """Where the collider thread sits: its current syscall (or 'running')
    every 20 ms, as a histogram per collider phase."""
    hist = {}
    path = '/proc/self/task/%d/syscall' % tid
    while not stop.is_set():
        try:
            with open(path) as f:
                word = f.read().split()
            key = 'running' if not word or word[0] == 'running' else \
                'sys_%s' % word[0]
        except OSError:
            key = 'gone'
        phase = out.get('_phase', 'pre')
        bucket = hist.setdefault(phase, {})
        bucket[key] = bucket.get(key, 0) + 1
        time.sleep(0.02)
    out['syscalls'] = hist


def collide(mod, out, delay_s):
    """The node agent's first generation, phase by phase."""
    time.sleep(delay_s)
    stop = threading.Event()
    sampler = threading.Thread(target=sample_syscalls, args=(
        threading.get_native_id(), out, stop), daemon=True)
    sampler.start()
    out['_phase'] = 'uid'
    t = [time.monotonic_ns()]
    uid = mod.fence_unique_id()
    t.append(time.monotonic_ns())
    out['_phase'] = 'init'
    fence = mod.Fence(uid, 1, 0, 60.0)
    t.append(time.monotonic_ns())
    out['_phase'] = 'allreduce'
    fence.allreduce([1] * 9)
    t.append(time.monotonic_ns())
    out['_phase'] = 'destroy'
    fence.destroy()
    t.append(time.monotonic_ns())
    stop.set()
    sampler.join()
    out.pop('_phase', None)
    out['done'] = True
    out['phases'] = {name: [t[i], t[i + 1]] for i, name in enumerate(PHASES)}


def sidecar_main():
    os.environ.setdefault('NCCL_MIN_NCHANNELS', '1')
    os.environ.setdefault('NCCL_MAX_NCHANNELS', '1')
    from kiosk_autoscaler_amd.ops import native
    mod = native.load(torch_first=False)
    mod.preinit_device(0)
    sys.stdout.write('ready\n')
    sys.stdout.flush()
    sys.stdin.readline()           # go
    out = {}
    collide(mod, out, 0.0)
    sys.stdout.write(json.dumps(out) + '\n')
    sys.stdout.flush()


def child_main(collider, work, seconds):
    os.environ.setdefault('NCCL_MIN_NCHANNELS', '1')
    os.environ.setdefault('NCCL_MAX_NCHANNELS', '1')
    side = None
    if collider == 'sidecar':
        # started before this process touches the GPU (no fork of a
        # process with a HIP context)
        side = subprocess.Popen(
            [sys.executable, __file__, '--sidecar'], stdin=subprocess.PIPE,
            stdout=subprocess.PIPE, text=True, env=dict(os.environ))
    from kiosk_autoscaler_amd.ops import native
    mod = native.load(torch_first=False)
    mod.preinit_device(0)
    engine = mod.Engine(0, 4096, 16384, 4, 2048, 1)
    engine.warmstart()
    for _ in range(5):
        engine.forward(2048, 1, 0)
    if side is not None:
        while side.stdout.readline().strip() != 'ready':
            if side.poll() is not None:
                raise RuntimeError('sidecar exited before ready')
    coll = {}
    thread = None
    t_go = time.monotonic_ns()
    if collider == 'inproc':
        thread = threading.Thread(target=collide, args=(mod, coll, 0.2))
        thread.start()
    elif collider == 'sidecar':
        time.sleep(0.2)
        side.stdin.write('go\n')
        side.stdin.flush()
    calls = []
    deadline = time.monotonic() + seconds
    hard = time.monotonic() + 150.0
    build_engine = None
    side_line = []
    if side is not None:
        def read_side():
            for line in side.stdout:
                if line.startswith('{'):
                    side_line.append(line)
        reader = threading.Thread(target=read_side, daemon=True)
        reader.start()

    def collider_done():
        if collider == 'inproc':
            return not thread.is_alive()
        if collider == 'sidecar':
            return bool(side_line)
        return True
    # keep working until the collider has finished every phase (+ 0.3 s)
    done_at = None
    while time.monotonic() < hard:
        now = time.monotonic()
        if done_at is None and collider_done():
            done_at = now
        if now >= deadline and done_at is not None and now - done_at > 0.3:
            break
        t0 = time.monotonic_ns()
        if work == 'forward':
            engine.forward(2048, 1, 0)
        elif work == 'ready':
            engine.warmstart()
        else:
            if build_engine is not None:
                build_engine.close()
            build_engine = mod.Engine(0, 4096, 16384, 4, 2048, 2)
            build_engine.warmstart()
            build_engine.forward(2048, 1, 0)
        t1 = time.monotonic_ns()
        calls.append((t0, t1))
    if build_engine is not None:
        build_engine.close()
    if thread is not None:
        thread.join()
    if side is not None:
        side.wait(timeout=60)
        coll = json.loads(side_line[-1]) if side_line else \
            {'error': 'no sidecar result'}
    engine.close()
    walls = sorted((b - a) / 1e6 for a, b in calls)
    row = {'collider': collider, 'work': work, 'calls': len(calls),
           'median_ms': round(walls[len(walls) // 2], 3) if walls else None,
           'max_ms': round(walls[-1], 3) if walls else None,
           'go_ns': t_go}
    phases = coll.get('phases') or {}
    row['phase_ms'] = {k: round((v[1] - v[0]) / 1e6, 1)
                       for k, v in phases.items()}
    overlap = {}
    for name, (p0, p1) in phases.items():
        hit = sorted((b - a) / 1e6 for a, b in calls if a < p1 and b > p0)
        if hit:
            overlap[name] = {'n': len(hit),
                             'median_ms': round(hit[len(hit) // 2], 3),
                             'max_ms': round(hit[-1], 3)}
    row['overlap'] = overlap
    row['syscalls'] = coll.get('syscalls')
    # the worst call and what it overlapped
    if calls:
        a, b = max(calls, key=lambda c: c[1] - c[0])
        row['worst_call'] = {
            'ms': round((b - a) / 1e6, 3),
            'overlaps': [n for n, (p0, p1) in phases.items()
                         if a < p1 and b > p0]}
    print(json.dumps(row), flush=True)


def main():
    if '--sidecar' in sys.argv:
        sidecar_main()
        return 0
    parser = argparse.ArgumentParser()
    parser.add_argument('--child', action='store_true')
    parser.add_argument('--collider', default='inproc')
    parser.add_argument('--work', default='forward')
    parser.add_argument('--seconds', type=float, default=6.0)
    parser.add_argument('--modes', default='none:forward,inproc:forward,'
                        'sidecar:forward,none:build,inproc:build,'
                        'sidecar:build')
    parser.add_argument('--out', default='')
    parser.add_argument('--debug-dir', default='',
                        help='RCCL INFO log with timestamps per mode')
    args = parser.parse_args()
    if args.child:
        child_main(args.collider, args.work, args.seconds)
        return 0
    rc = 0
    sink = open(args.out, 'a') if args.out else None
    for mode in args.modes.split(','):
        collider, work = mode.split(':')
        env = dict(os.environ)
        if args.debug_dir:
            os.makedirs(args.debug_dir, exist_ok=True)
            env.update({'NCCL_DEBUG': 'INFO',
                        'NCCL_DEBUG_SUBSYS': 'INIT,BOOTSTRAP,NET,ENV,ALLOC',
                        'NCCL_DEBUG_TIMESTAMP_LEVELS': 'ALL',
                        'NCCL_DEBUG_FILE': os.path.join(
                            args.debug_dir, '%s_%s.%%p.log' % (collider,
                                                                work))})
        proc = subprocess.run(
            [sys.executable, __file__, '--child', '--collider', collider,
             '--work', work, '--seconds', str(args.seconds)],
            capture_output=True, text=True, timeout=240, env=env)
        line = proc.stdout.strip().splitlines()[-1] if proc.stdout.strip() \
            else json.dumps({'collider': collider, 'work': work,
                             'rc': proc.returncode,
                             'stderr': proc.stderr[-1500:]})
        print(line, flush=True)
        if sink:
            sink.write(line + '\n')
            sink.flush()
        if proc.returncode:
            rc = proc.returncode
            break
    return rc


if __name__ == '__main__':
    sys.exit(main())
