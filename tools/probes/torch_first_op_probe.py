#!/usr/bin/env python3
"""Which torch call pays torch's one-time GPU set-up in a PyTorch standby?

After ``warm_device`` stopped launching a torch fill kernel, the engine
build's forward capture grew from 0.4 to 11.8 ms (``profiles/r4_comgr``):
some torch state is set up on the first real GPU operation.  Each child
(fresh process, the worker's load order and ``preinit_device``) runs the
engine build's torch operations one by one in a given order, each twice,
and prints the ms of every call.  The parent never touches the GPU.

    python tools/torch_first_op_probe.py
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ORDERS = ['h2d,graph,d2h,event', 'graph,h2d,d2h,event',
          'event,h2d,graph,d2h', 'd2h,h2d,graph,event']


def child(order):
    sys.path.insert(0, ROOT)
    from kiosk_autoscaler_amd.ops import native
    mod = native.load(torch_first=True)
    import torch
    mod.preinit_device(0)
    torch.cuda.init()
    mod.prepare_kernels()
    handle = mod.take_stream(0)
    stream = torch.cuda.ExternalStream(handle, device=torch.device('cuda'))
    from torch.utils.dlpack import from_dlpack
    arena = from_dlpack(mod.device_buffer(1 << 20, 0))
    dev = arena[:64].view(torch.int64)
    host = torch.zeros(8, dtype=torch.int64).pin_memory()
    host_out = torch.zeros(8, dtype=torch.int64).pin_memory()

    def h2d():
        with torch.cuda.stream(stream):
            dev[:8].copy_(host, non_blocking=True)
        stream.synchronize()

    def d2h():
        with torch.cuda.stream(stream):
            host_out.copy_(dev[:8], non_blocking=True)
        stream.synchronize()

    def graph():
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(stream):
            g.capture_begin(capture_error_mode='thread_local')
            mod.memset_async(dev.data_ptr(), 0, 64, stream.cuda_stream)
            g.capture_end()
        g.replay()
        stream.synchronize()

    def event():
        e = torch.cuda.Event()
        e.record(stream)
        e.synchronize()

    ops = {'h2d': h2d, 'd2h': d2h, 'graph': graph, 'event': event}
    row = {'order': order}
    for rnd in (1, 2):
        for name in order.split(','):
            t0 = time.perf_counter()
            ops[name]()
            row['%s_%d' % (name, rnd)] = round(
                (time.perf_counter() - t0) * 1e3, 3)
    mod.return_stream(handle, 0)
    print(json.dumps(row), flush=True)


def main():
    if len(sys.argv) > 2 and sys.argv[1] == '--child':
        child(sys.argv[2])
        return 0
    for _ in range(2):
        for order in ORDERS:
            out = subprocess.run([sys.executable, os.path.abspath(__file__),
                                  '--child', order], stdout=subprocess.PIPE,
                                 timeout=120, check=True)
            sys.stdout.write(out.stdout.decode())
            sys.stdout.flush()
    return 0


if __name__ == '__main__':
    sys.exit(main())
