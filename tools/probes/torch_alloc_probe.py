#!/usr/bin/env python3
"""Why does a PyTorch engine's 1.2 GB arena take ~115 ms to allocate when
the built-in engine's takes under 1 ms (``tools/torch_boot_probe.py``)?

Each row is a fresh child process: import torch, open the device through
the native module (``preinit_device``) and torch, then time

* ``native_engine``: the built-in ``Engine`` (its own ``hipMalloc`` arena)
  in this torch process -- the HIP runtime is torch's either way;
* ``torch_empty``: ``torch.empty`` of the arena's size, cold and again
  after freeing it (the caching allocator then reuses the segment);
* the same under ``PYTORCH_HIP_ALLOC_CONF=expandable_segments:True``.

    python tools/torch_alloc_probe.py
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
NBYTES = 1_207_959_552 + 64 * 1024 * 1024


def child(order):
    import torch
    sys.path.insert(0, ROOT)
    from kiosk_autoscaler_amd.ops import native
    mod = native.load()
    mod.preinit_device(0)
    torch.empty(1, device='cuda').zero_()
    torch.cuda.synchronize()
    row = {'order': order,
           'alloc_conf': os.environ.get('PYTORCH_HIP_ALLOC_CONF', '')}

    def timed(name, fn):
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        row[name] = round((time.perf_counter() - t0) * 1e3, 2)
        return out
    for step in order.split(','):
        if step == 'native':
            engine = timed('native_engine_ms',
                           lambda: mod.Engine(0, 4096, 16384, 4, 2048, 1))
            engine.close()
        elif step == 'dlpack':
            from torch.utils.dlpack import from_dlpack
            free0 = mod.mem_info()[0]
            t = timed('dlpack_buffer_ms',
                      lambda: from_dlpack(mod.device_buffer(NBYTES, 0)))
            row['dlpack_ok'] = (t.is_cuda and t.numel() == NBYTES and
                                t.dtype == torch.uint8)
            t[:16].fill_(7)
            row['dlpack_fill_ok'] = int(t[:16].sum()) == 7 * 16
            held = free0 - mod.mem_info()[0]
            del t
            torch.cuda.synchronize()
            row['dlpack_held_mib'] = round(held / 2 ** 20)
            row['dlpack_freed_mib'] = round((mod.mem_info()[0] - free0 +
                                             held) / 2 ** 20)
            # never consumed: the capsule's own destructor frees it
            cap = mod.device_buffer(1 << 20, 0)
            del cap
        elif step == 'torch':
            t = timed('torch_empty_ms', lambda: torch.empty(
                NBYTES, dtype=torch.uint8, device='cuda'))
            del t
            t = timed('torch_empty_reuse_ms', lambda: torch.empty(
                NBYTES, dtype=torch.uint8, device='cuda'))
            del t
            torch.cuda.empty_cache()
            t = timed('torch_empty_after_release_ms', lambda: torch.empty(
                NBYTES, dtype=torch.uint8, device='cuda'))
            del t
            t = timed('torch_empty_64MiB_ms', lambda: torch.empty(
                64 << 20, dtype=torch.uint8, device='cuda'))
            del t
    print(json.dumps(row), flush=True)


def main():
    if len(sys.argv) > 2 and sys.argv[1] == '--child':
        child(sys.argv[2])
        return 0
    runs = [('native,torch', ''), ('dlpack,torch,native', ''),
            ('torch', 'expandable_segments:True')]
    for order, conf in runs:
        env = dict(os.environ)
        if conf:
            env['PYTORCH_HIP_ALLOC_CONF'] = conf
        out = subprocess.run([sys.executable, os.path.abspath(__file__),
                              '--child', order], env=env,
                             stdout=subprocess.PIPE, timeout=240, check=True)
        sys.stdout.write(out.stdout.decode())
        sys.stdout.flush()
    return 0


if __name__ == '__main__':
    sys.exit(main())
