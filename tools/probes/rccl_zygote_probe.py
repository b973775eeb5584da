#!/usr/bin/env python3
"""Can the worker zygote pay RCCL's fat-binary registration once for every
worker it forks?

The parent never touches the GPU (like the zygote).  With ``--preload`` it
dlopens RCCL first (``_kiosk_hip.fence_dlopen``: the library's static
constructors register its fat binary; no HIP call).  Then it forks a child
that does what a woken standby does -- open the device, build the engine,
time a warm-start graph -- and then what its node agent does: RCCL library
init (``fence_preload``), a 1-rank communicator, a 72-B all-reduce.  One
JSON line per child: the stage times in ms and the child's thread count
after the fork (a registration that spawned threads would not survive
``fork``).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def child(out_fd, preloaded):
    os.environ.setdefault('NCCL_MIN_NCHANNELS', '1')
    os.environ.setdefault('NCCL_MAX_NCHANNELS', '1')
    from kiosk_autoscaler_amd.ops import native
    row = {'preloaded_in_parent': preloaded,
           'threads_after_fork': len(os.listdir('/proc/self/task'))}
    t = time.perf_counter()
    mod = native.load(torch_first=False)
    mod.preinit_device(0)
    row['preinit_ms'] = (time.perf_counter() - t) * 1e3
    t = time.perf_counter()
    engine = mod.Engine(0, 4096, 16384, 4, 2048, 1)
    engine.warmstart()
    row['engine_ms'] = (time.perf_counter() - t) * 1e3
    t = time.perf_counter()
    engine.warmstart()
    row['ready_ms'] = (time.perf_counter() - t) * 1e3
    t = time.perf_counter()
    row['fence_preload_ms'] = mod.fence_preload()
    row['fence_preload_wall_ms'] = (time.perf_counter() - t) * 1e3
    t = time.perf_counter()
    fence = mod.Fence(mod.fence_unique_id(), 1, 0, 60.0)
    row['comm_init_ms'] = (time.perf_counter() - t) * 1e3
    result, us = fence.allreduce([1] * 9)
    row['allreduce_ok'] = list(result) == [1] * 9
    row['allreduce_us'] = us
    t = time.perf_counter()
    fence.destroy()
    row['destroy_ms'] = (time.perf_counter() - t) * 1e3
    engine.close()
    os.write(out_fd, (json.dumps(row) + '\n').encode())


def main():
    preload = '--preload' in sys.argv
    from kiosk_autoscaler_amd.ops import native
    mod = native.load(torch_first=False)
    parent = {'parent_threads_before': len(os.listdir('/proc/self/task'))}
    if preload:
        t = time.perf_counter()
        mod.fence_dlopen()
        parent['parent_dlopen_ms'] = (time.perf_counter() - t) * 1e3
    parent['parent_threads_after'] = len(os.listdir('/proc/self/task'))
    r, w = os.pipe()
    pid = os.fork()
    if pid == 0:
        os.close(r)
        code = 0
        try:
            child(w, preload)
        except BaseException as err:  # pylint: disable=broad-except
            os.write(w, (json.dumps({'error': repr(err)}) + '\n').encode())
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
    row = json.loads(data.decode().strip().splitlines()[-1]) if data else {}
    row.update(parent)
    row['child_status'] = os.waitstatus_to_exitcode(status)
    print(json.dumps(row), flush=True)
    return 0 if row.get('child_status') == 0 else 1


if __name__ == '__main__':
    sys.exit(main())
