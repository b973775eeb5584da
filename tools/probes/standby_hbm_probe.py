"""Probe: device VRAM (amdsmi) a worker process holds after each start-up
stage -- HIP context + code objects (preinit), the 1-rank node
communicator (RCCL, 1 channel as the worker sets it), the engine (arena,
weights, captured graph) and after releasing each -- to see what a standby
holds and what it could give back.  One JSON line per stage."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ.setdefault('NCCL_MIN_NCHANNELS', '1')
os.environ.setdefault('NCCL_MAX_NCHANNELS', '1')


def main():
    import amdsmi
    amdsmi.amdsmi_init()
    handle = amdsmi.amdsmi_get_processor_handles()[0]

    def used():
        time.sleep(0.3)
        return amdsmi.amdsmi_get_gpu_vram_usage(handle)['vram_used']
    # a previous tenant's memory may still be draining: wait until stable
    base = used()
    deadline = time.monotonic() + 60
    while time.monotonic() < deadline:
        time.sleep(1.0)
        now = used()
        if abs(now - base) <= 16:
            break
        base = now
    rows = []
    mod = None

    def mark(stage):
        value = used()
        row = {'stage': stage, 'vram_used_mib': value,
               'over_start_mib': value - base}
        if mod is not None:
            free, total = mod.mem_info()
            row['hip_used_mib'] = (total - free) / 2 ** 20
        rows.append(row)
        print(json.dumps(row), flush=True)
    mark('start (stable)')
    from kiosk_autoscaler_amd.ops import native
    mod = native.load()
    mark('HIP context (hipMemGetInfo)')
    stages = mod.preload_modules(0)
    mark('code objects loaded without a launch (context standby, %.1f ms)'
         % ((stages['preload_done'] - stages['preload_context']) / 1e6))
    mod.preinit_device(0)
    mark('preinit (code objects, one launch of each kernel)')
    fence = mod.Fence(1, 0, 30.0)
    fence.connect(mod.fence_unique_id())
    fence.allreduce([1, 1])
    mark('node communicator (RCCL, 1 rank, 1 channel)')
    engine = mod.Engine(0, 4096, 16384, 4, 2048, 1234)
    engine.prepare(2048)
    engine.forward(2048, 1, 7)
    mod.synchronize()
    mark('engine (arena, weights, graph) after one forward')
    engine.close()
    mod.synchronize()
    mark('engine closed')
    fence.destroy()
    mark('communicator destroyed')
    free, total = mod.mem_info()
    print(json.dumps({'hip_mem_info_free_mib': free / 2 ** 20,
                      'total_mib': total / 2 ** 20}), flush=True)
    amdsmi.amdsmi_shut_down()


if __name__ == '__main__':
    main()
