#!/usr/bin/env python3
"""How long a worker's exit holds its GPU: ``os._exit`` -> reaped, by what
the process holds (the tail of every deep-idle cycle: a parked standby's
exit is standby GPU time, profiles/r5_standby).

Like the zygote, the parent loads the native module (and RCCL, and torch
for the ``torch`` cases) without a HIP call and forks one child per case;
the child builds what the case names, reports, waits for ``go`` and calls
``os._exit``; the parent times ``go`` -> ``waitpid``.

Cases: ``ctx`` (HIP context + stream), ``engine`` (+ the production engine,
1.3 GB), ``engine_rccl`` (+ a 1-rank RCCL communicator), ``engine_free``
(engine closed -- hipFree -- before the exit, timed separately),
``torch_engine_rccl`` (the PyTorch engine + RCCL), ``engine_rccl_abort`` /
``engine_rccl_destroy`` (the communicator aborted / destroyed after ``go``,
before the exit; ``teardown_ms``), ``rccl`` (context + communicator, no
engine).  One JSON line per case; ``EXIT_PROBE_TAG`` is copied into it
(environment variants of one case, run one process each).
``torch_engine_rccl_reset`` / ``_hsashut``: ``hipDeviceReset`` /
``hsa_shut_down`` after ``go``, before the exit (does a user-space
teardown shorten the kernel's?).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

CASES = ('ctx', 'engine', 'engine_rccl', 'engine_free', 'torch_engine_rccl',
         'engine_rccl_abort', 'engine_rccl_destroy', 'rccl', 'streams_2',
         'streams_hi_2', 'torch_engine_rccl_reset', 'torch_engine_rccl_hsashut')


def child(case, mod, wfd, rfd):
    info = {}
    mod.preinit_device(0)
    keep = []
    if case.startswith('torch'):
        from kiosk_autoscaler_amd.models.torch_kiosk import TorchKioskEngine
        from kiosk_autoscaler_amd.worker.runtime import WorkerConfig
        cfg = WorkerConfig({'MODEL_DIM': '4096', 'MODEL_HIDDEN': '16384',
                            'MODEL_LAYERS': '4', 'ROWS_PER_KEY': '2048'},
                           {'worker_id': 'exit'})
        engine = TorchKioskEngine(cfg)
        engine.warmstart()
        keep.append(engine)
    elif case.startswith('engine'):
        engine = mod.Engine(0, 4096, 16384, 4, 2048, 1)
        engine.warmstart()
        keep.append(engine)
    if case.startswith('streams'):
        # ``streamsN`` / ``streams_hiN``: N more HIP streams, each used once
        # (a hardware queue is made at a stream's first use), at normal or
        # high priority -- does the exit scale with the queues?
        import ctypes
        hip = ctypes.CDLL('libamdhip64.so', mode=ctypes.RTLD_GLOBAL)
        n = int(case.rstrip('_').split('_')[-1].lstrip('streamshi') or 1)
        buf = ctypes.c_void_p()
        hip.hipMalloc(ctypes.byref(buf), ctypes.c_size_t(1 << 20))
        for _ in range(n):
            stream = ctypes.c_void_p()
            if '_hi' in case:
                hip.hipStreamCreateWithPriority(ctypes.byref(stream), 0, -1)
            else:
                hip.hipStreamCreate(ctypes.byref(stream))
            hip.hipMemsetAsync(buf, 0, ctypes.c_size_t(1 << 20), stream)
            hip.hipStreamSynchronize(stream)
            keep.append(stream)
    if 'rccl' in case:
        free, total = mod.mem_info()
        before = total - free
        t0 = time.monotonic_ns()
        fence = mod.Fence(mod.fence_unique_id(), 1, 0, 60.0)
        fence.allreduce([1] * 9)
        info['rccl_init_ms'] = (time.monotonic_ns() - t0) / 1e6
        free, total = mod.mem_info()
        info['rccl_hbm_mb'] = (total - free - before) / 1e6
        keep.append(fence)
    if case.endswith(('_abort', '_destroy', '_reset', '_hsashut')):
        # timed in the child just before its exit: what the comm's own
        # teardown costs against the kernel's at exit
        info['teardown'] = case.rsplit('_', 1)[1]
    if case == 'engine_free':
        t0 = time.monotonic_ns()
        keep[0].close()
        info['close_ms'] = (time.monotonic_ns() - t0) / 1e6
    free, total = mod.mem_info()
    info['used_gb'] = (total - free) / 1e9
    os.write(wfd, (json.dumps(info) + '\n').encode())
    os.read(rfd, 1)            # go
    if 'teardown' in info:
        t0 = time.monotonic_ns()
        if info['teardown'] == 'reset':
            # the HIP runtime frees its device state in user space first
            import ctypes
            ctypes.CDLL('libamdhip64.so').hipDeviceReset()
        elif info['teardown'] == 'hsashut':
            # ROCr's own teardown (queues, signals, memory) before the exit
            import ctypes
            ctypes.CDLL('libhsa-runtime64.so.1').hsa_shut_down()
        else:
            getattr(keep[-1], info['teardown'])()
        os.write(wfd, ('%.3f\n' % ((time.monotonic_ns() - t0) / 1e6)).encode())
    os._exit(0)


def _threads(pid):
    try:
        return len(os.listdir('/proc/%d/task' % pid))
    except OSError:
        return None


def _memory(pid):
    """The child's mappings before its exit: what ``exit_mm`` tears down."""
    out = {}
    try:
        with open('/proc/%d/status' % pid) as f:
            for line in f:
                key, _, value = line.partition(':')
                if key in ('VmRSS', 'RssAnon', 'RssFile', 'RssShmem',
                           'VmPin', 'VmLck', 'VmSize'):
                    out[key + '_mb'] = round(int(value.split()[0]) / 1024.0)
        with open('/proc/%d/maps' % pid) as f:
            out['maps'] = sum(1 for _ in f)
    except (OSError, ValueError):
        pass
    return out


def _smaps(pid, top=10):
    """``EXIT_PROBE_SMAPS=1``: the child's largest anonymous mappings
    (what its exit frees page by page), with their THP share."""
    rows = []
    cur = None
    try:
        with open('/proc/%d/smaps' % pid) as f:
            for line in f:
                parts = line.split()
                if '-' in parts[0] and not parts[0].endswith(':'):
                    lo, hi = (int(x, 16) for x in parts[0].split('-'))
                    cur = {'name': parts[5] if len(parts) > 5 else '[anon]',
                           'perm': parts[1], 'size_mb': (hi - lo) >> 20,
                           'anon_mb': 0, 'thp_mb': 0}
                    rows.append(cur)
                elif parts[0] == 'Anonymous:' and cur is not None:
                    cur['anon_mb'] = int(parts[1]) >> 10
                elif parts[0] == 'AnonHugePages:' and cur is not None:
                    cur['thp_mb'] = int(parts[1]) >> 10
    except OSError:
        return None
    rows.sort(key=lambda r: -r['anon_mb'])
    total = sum(r['anon_mb'] for r in rows)
    return {'anon_mb': total, 'mappings': len(rows), 'top': rows[:top]}


KFD_PROC = '/sys/class/kfd/kfd/proc/%d'


def _kfd_dirs():
    try:
        return set(os.listdir(os.path.dirname(KFD_PROC)))
    except OSError:
        return set()


def _wait_sampling(pid, t0=None, info=None):
    """``waitpid`` by polling, sampling every 0.5 ms where the exiting
    process's threads sleep in the kernel (``/proc/<pid>/task/*/wchan`` and
    the thread state, readable by the owner): ``{state:wchan: samples}``.
    With ``info``: ``kfd_gone_ms``, ``t0`` -> the instant the process's KFD
    record (``/sys/class/kfd/kfd/proc/<pid>``, removed once the driver has
    torn down its queues and GPU memory) disappeared."""
    import collections
    where = collections.Counter()
    # the record is named by the host's PID, not this namespace's: the
    # caller passes the directory that appeared while the child started
    kfd = (info or {}).pop('_kfd_dir', None) or KFD_PROC % pid
    watch = info is not None and os.path.exists(kfd)
    if info is not None:
        info['kfd_record'] = watch
    while True:
        if watch and not os.path.exists(kfd):
            info['kfd_gone_ms'] = (time.monotonic_ns() - t0) / 1e6
            watch = False
        done, status = os.waitpid(pid, os.WNOHANG)
        if done:
            if info is not None:
                info['reaped_ms'] = (time.monotonic_ns() - t0) / 1e6
            if watch and not os.path.exists(kfd):
                info['kfd_gone_ms'] = (time.monotonic_ns() - t0) / 1e6
            elif watch:
                # still there when reaped: the driver's release work runs
                # after the process (poll up to 0.5 s more)
                info['kfd_after_reap'] = True
                end = time.monotonic() + 0.5
                while os.path.exists(kfd) and time.monotonic() < end:
                    time.sleep(0.0005)
                info['kfd_gone_ms'] = ((time.monotonic_ns() - t0) / 1e6
                                       if not os.path.exists(kfd) else None)
            return status, dict(where.most_common(12))
        try:
            tids = os.listdir('/proc/%d/task' % pid)
        except OSError:
            tids = []
        for tid in tids:
            base = '/proc/%d/task/%s/' % (pid, tid)
            try:
                with open(base + 'stat') as f:
                    state = f.read().rsplit(')', 1)[1].split()[0]
                with open(base + 'wchan') as f:
                    chan = f.read().strip() or '-'
            except OSError:
                continue
            where['%s:%s' % (state, chan)] += 1
        time.sleep(0.0005)


def main():
    cases = sys.argv[1].split(',') if len(sys.argv) > 1 else list(CASES)
    os.environ.setdefault('NCCL_MIN_NCHANNELS', '1')
    os.environ.setdefault('NCCL_MAX_NCHANNELS', '1')
    torch_first = any(c.startswith('torch') for c in cases)
    if os.environ.get('EXIT_PROBE_SLIM') == '1':
        # the one-ISA RCCL copy the manager writes (what workers load)
        from kiosk_autoscaler_amd.parallel import rccl_lib
        print(json.dumps({'rccl_lib': rccl_lib.configure()}), flush=True)
    from kiosk_autoscaler_amd.ops import native
    mod = native.load(torch_first=torch_first)
    mod.fence_dlopen()
    for case in cases:
        for rep in range(3):
            up_r, up_w = os.pipe()
            go_r, go_w = os.pipe()
            kfd_before = _kfd_dirs()
            pid = os.fork()
            if pid == 0:
                os.close(up_r)
                os.close(go_w)
                try:
                    child(case, mod, up_w, go_r)
                except Exception as err:  # pylint: disable=broad-except
                    os.write(up_w, (json.dumps({'error': str(err)}) +
                                    '\n').encode())
                    os._exit(1)
            os.close(up_w)
            os.close(go_r)
            line = b''
            while not line.endswith(b'\n'):
                chunk = os.read(up_r, 4096)
                if not chunk:
                    break
                line += chunk
            info = json.loads(line.decode() or '{}')
            fresh = sorted(_kfd_dirs() - kfd_before)
            info['kfd_new_records'] = len(fresh)
            if len(fresh) == 1:
                info['_kfd_dir'] = os.path.join(os.path.dirname(KFD_PROC),
                                                fresh[0])
            time.sleep(0.2)
            threads = _threads(pid)
            info['mem'] = _memory(pid)
            if os.environ.get('EXIT_PROBE_SMAPS') == '1':
                info['smaps'] = _smaps(pid)
            t0 = time.monotonic_ns()
            os.write(go_w, b'g')
            status, where = _wait_sampling(pid, t0, info)
            if 'teardown' in info:
                tail = os.read(up_r, 64).decode().strip()
                info['teardown_ms'] = float(tail) if tail else None
            info.update({'threads': threads, 'where': where})
            info.update({'case': case, 'rep': rep,
                         'tag': os.environ.get('EXIT_PROBE_TAG', ''),
                         'exit_ms': (time.monotonic_ns() - t0) / 1e6,
                         'status': status})
            print(json.dumps(info), flush=True)
            os.close(up_r)
            os.close(go_w)
            if os.WIFSIGNALED(status):
                # a child that died by a signal: nothing more on the GPU
                print(json.dumps({'stopped': case, 'signal':
                                  os.WTERMSIG(status)}), flush=True)
                return 3
            time.sleep(0.3)
    return 0


if __name__ == '__main__':
    sys.exit(main())
