#!/usr/bin/env python3
"""Where a fresh worker's first node-communicator generation spends its time
(READY -> fenced took 1.75 s).

Each case runs in its own process tree, shaped like production: a parent
that loads the native module and ``dlopen``s RCCL *before any HIP call* (the
worker zygote, ``worker/zygote.py``), then forks a child that opens the
device, builds the production engine (4 x 4096->16384->4096, 2048 rows) and
times the node agent's first generation: ``ncclGetUniqueId`` ->
``ncclCommInitRank`` (1 rank) -> 72-B all-reduce -> destroy, then a second
generation in the same process.  With ``serving`` the main thread keeps
launching forwards meanwhile, as a worker serving its first key does.

Cases: ``--libs stock,slim`` (ROCm's librccl vs the one-ISA copy of
``parallel/rccl_lib.py``) x ``--scenarios idle,serving``.  RCCL's INFO log
(``Init timings`` per phase) goes to ``--debug-dir``.  One JSON line per
case on stdout.
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def generation(mod):
    t = [time.monotonic_ns()]
    uid = mod.fence_unique_id()
    t.append(time.monotonic_ns())
    fence = mod.Fence(uid, 1, 0, 60.0)
    t.append(time.monotonic_ns())
    result, us = fence.allreduce([1] * 9)
    t.append(time.monotonic_ns())
    fence.destroy()
    t.append(time.monotonic_ns())
    names = ('uid', 'init', 'allreduce', 'destroy')
    out = {n: round((t[i + 1] - t[i]) / 1e6, 2) for i, n in enumerate(names)}
    out['total'] = round((t[-1] - t[0]) / 1e6, 2)
    out['ok'] = list(result) == [1] * 9
    return out


def child(mod, scenario, wfd):
    row = {}
    t0 = time.monotonic_ns()
    mod.preinit_device(0)
    row['preinit_ms'] = round((time.monotonic_ns() - t0) / 1e6, 2)
    engine = mod.Engine(0, 4096, 16384, 4, 2048, 1)
    engine.warmstart()
    for _ in range(3):
        engine.forward(2048, 1, 0)
    stop = threading.Event()
    calls = []

    def serve():
        while not stop.is_set():
            a = time.monotonic_ns()
            engine.forward(2048, 1, 0)
            calls.append((time.monotonic_ns() - a) / 1e6)
    thread = None
    if scenario == 'serving':
        thread = threading.Thread(target=serve, daemon=True)
        thread.start()
        time.sleep(0.05)
    row['first'] = generation(mod)
    row['second'] = generation(mod)
    stop.set()
    if thread is not None:
        thread.join()
        calls.sort()
        row['forward_calls'] = len(calls)
        row['forward_median_ms'] = round(calls[len(calls) // 2], 3) \
            if calls else None
        row['forward_max_ms'] = round(calls[-1], 3) if calls else None
    engine.close()
    os.write(wfd, (json.dumps(row) + '\n').encode())


def case(lib, scenario):
    """One case in this process (the zygote's role) + a forked child."""
    from kiosk_autoscaler_amd.ops import native
    mod = native.load(torch_first=False)
    t0 = time.monotonic_ns()
    mod.fence_dlopen()
    dlopen_ms = (time.monotonic_ns() - t0) / 1e6
    r, w = os.pipe()
    pid = os.fork()
    if pid == 0:
        os.close(r)
        code = 0
        try:
            child(mod, scenario, w)
        except Exception as err:  # pylint: disable=broad-except
            os.write(w, (json.dumps({'error': str(err)}) + '\n').encode())
            code = 1
        os._exit(code)
    os.close(w)
    data = b''
    while True:
        chunk = os.read(r, 65536)
        if not chunk:
            break
        data += chunk
    _, status = os.waitpid(pid, 0)
    row = json.loads(data.decode().strip() or '{}')
    row.update({'lib': lib, 'scenario': scenario,
                'rccl': os.environ.get('KIOSK_RCCL_LIB'),
                'dlopen_ms': round(dlopen_ms, 2), 'status': status})
    print(json.dumps(row), flush=True)


def main():
    import subprocess
    parser = argparse.ArgumentParser()
    parser.add_argument('--case', default='')
    parser.add_argument('--libs', default='stock,slim')
    parser.add_argument('--scenarios', default='idle,serving')
    parser.add_argument('--debug-dir', default='')
    parser.add_argument('--out', default='')
    args = parser.parse_args()
    if args.case:
        lib, scenario = args.case.split(':')
        case(lib, scenario)
        return 0
    from kiosk_autoscaler_amd.parallel import rccl_lib
    slim, info = rccl_lib.ensure_slim()
    print(json.dumps({'slim': slim, 'info': info}), flush=True)
    sink = open(args.out, 'a') if args.out else None
    rc = 0
    for lib in args.libs.split(','):
        for scenario in args.scenarios.split(','):
            env = dict(os.environ)
            env['NCCL_MIN_NCHANNELS'] = env['NCCL_MAX_NCHANNELS'] = '1'
            env['KIOSK_RCCL_LIB'] = rccl_lib.STOCK if lib == 'stock' else \
                (slim or rccl_lib.STOCK)
            if args.debug_dir:
                os.makedirs(args.debug_dir, exist_ok=True)
                env.update({'NCCL_DEBUG': 'INFO',
                            'NCCL_DEBUG_SUBSYS': 'INIT',
                            'NCCL_DEBUG_FILE': os.path.join(
                                args.debug_dir, '%s_%s.%%p.log' % (
                                    lib, scenario))})
            proc = subprocess.run(
                [sys.executable, __file__, '--case', '%s:%s' % (lib, scenario)],
                capture_output=True, text=True, timeout=180, env=env)
            line = proc.stdout.strip().splitlines()[-1] if \
                proc.stdout.strip() else json.dumps({
                    'lib': lib, 'scenario': scenario, 'rc': proc.returncode,
                    'stderr': proc.stderr[-1500:]})
            print(line, flush=True)
            if sink:
                sink.write(line + '\n')
                sink.flush()
            if proc.returncode:
                rc = proc.returncode
                return rc
    return rc


if __name__ == '__main__':
    sys.exit(main())
