#!/usr/bin/env python3
"""Why does a process's first HIP stream cost 15-155 ms?

``profiles/r4_queue``: in a fresh process ``hipStreamCreateWithFlags`` took
91 ms (ROCm 7.2) and 155 ms (torch's bundled runtime), while every HSA call
inside it (``hsa_queue_create``, the pool allocations, the executable
freeze) adds up to about 15 ms.  The HIP runtime builds its blit kernels at
its first queue; this probe tests whether that build goes through comgr and
its on-disk cache (``AMD_COMGR_CACHE``, ``AMD_COMGR_CACHE_DIR``).

Each row is a fresh child that loads one runtime (``torch``: torch's bundled
``libamdhip64.so`` after ``import torch``; ``native``: ``/opt/rocm``'s) and
times ``hipFree(0)`` (context) and ``hipStreamCreate`` (first queue).  The
parent never touches the GPU.

    python tools/first_stream_probe.py --repeat 3
"""
import argparse
import ctypes
import json
import os
import shutil
import subprocess
import sys
import time


def child(kind):
    if kind == 'torch_rocm_comgr':
        # ROCm 7.2's comgr under torch's runtime (ops/native.py)
        ctypes.CDLL('libamd_comgr.so', mode=ctypes.RTLD_GLOBAL)
    if kind == 'torch_rocm_hsa':
        # ROCm 7.2's HSA runtime (and comgr) under torch's HIP runtime
        ctypes.CDLL('libhsa-runtime64.so', mode=ctypes.RTLD_GLOBAL)
        ctypes.CDLL('libamd_comgr.so', mode=ctypes.RTLD_GLOBAL)
    if kind.startswith('torch'):
        import torch
        lib = os.path.join(os.path.dirname(torch.__file__), 'lib',
                           'libamdhip64.so')
    else:
        lib = '/opt/rocm/lib/libamdhip64.so.7'
    hip = ctypes.CDLL(lib)
    t0 = time.perf_counter()
    rc = hip.hipFree(ctypes.c_void_p(0))
    t1 = time.perf_counter()
    stream = ctypes.c_void_p()
    rc2 = hip.hipStreamCreate(ctypes.byref(stream))
    t2 = time.perf_counter()
    rc3 = hip.hipStreamSynchronize(stream)
    # the process's first graph: capture one memset, instantiate, launch
    buf = ctypes.c_void_p()
    hip.hipMalloc(ctypes.byref(buf), ctypes.c_size_t(4096))
    graph_ms = []
    for _ in range(2):
        graph, exe = ctypes.c_void_p(), ctypes.c_void_p()
        g0 = time.perf_counter()
        hip.hipStreamBeginCapture(stream, 0)
        hip.hipMemsetAsync(buf, 0, ctypes.c_size_t(4096), stream)
        hip.hipStreamEndCapture(stream, ctypes.byref(graph))
        g1 = time.perf_counter()
        rc4 = hip.hipGraphInstantiate(ctypes.byref(exe), graph, None, None,
                                      ctypes.c_size_t(0))
        g2 = time.perf_counter()
        hip.hipGraphLaunch(exe, stream)
        hip.hipStreamSynchronize(stream)
        g3 = time.perf_counter()
        graph_ms.append([round((g1 - g0) * 1e3, 2), round((g2 - g1) * 1e3, 2),
                         round((g3 - g2) * 1e3, 2), rc4])
        hip.hipGraphExecDestroy(exe)
        hip.hipGraphDestroy(graph)
    hip.hipFree(buf)
    hip.hipStreamDestroy(stream)
    row = {'context_ms': round((t1 - t0) * 1e3, 2),
           'stream_ms': round((t2 - t1) * 1e3, 2), 'rc': [rc, rc2, rc3],
           'graph_capture_instantiate_launch_ms': graph_ms}
    if kind.startswith('torch'):
        # blit kernels (fill, copies) and a BLAS GEMM still work
        a = torch.full((512, 512), 0.5, device='cuda', dtype=torch.bfloat16)
        b = torch.arange(512 * 512, dtype=torch.float32).reshape(512, 512)
        b = b.to('cuda').to(torch.bfloat16) / 1e5
        c = (a @ b).float().cpu()
        ref = (a.float().cpu() @ b.float().cpu())
        row['torch_ops_ok'] = bool(torch.allclose(c, ref, rtol=2e-2,
                                                  atol=1e-2))
    with open('/proc/self/maps') as maps:
        row['comgr'] = sorted({line.split()[-1] for line in maps
                               if 'comgr' in line or 'hsa-runtime' in line})
    print(json.dumps(row), flush=True)


def cache_files(path):
    n = 0
    for _, _, files in os.walk(path):
        n += len(files)
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--child', choices=('torch', 'torch_rocm_comgr',
                                           'torch_rocm_hsa', 'native'))
    ap.add_argument('--kinds', default='native,torch,torch_rocm_comgr')
    ap.add_argument('--variants', default='default,cache_off,cache_dir')
    ap.add_argument('--repeat', type=int, default=3)
    ap.add_argument('--gap', type=float, default=0.0,
                    help='seconds between children (the previous one\'s '
                         'teardown)')
    ap.add_argument('--cache-root', default='/tmp/comgr_probe')
    args = ap.parse_args()
    if args.child:
        child(args.child)
        return 0
    home_cache = os.path.expanduser('~/.cache/comgr')
    print(json.dumps({'home_comgr_cache_before': os.path.isdir(home_cache),
                      'files': cache_files(home_cache)}), flush=True)
    variants = [('default', {}),
                ('cache_off', {'AMD_COMGR_CACHE': '0'}),
                ('cache_dir', {'AMD_COMGR_CACHE': '1',
                               'AMD_COMGR_CACHE_DIR': None}),
                ('no_packet_capture', {'DEBUG_CLR_GRAPH_PACKET_CAPTURE': '0'}),
                # context-creation knobs of the HSA runtime
                ('sdma_off', {'HSA_ENABLE_SDMA': '0'}),
                ('rocr_visible', {'ROCR_VISIBLE_DEVICES': '0'})]
    wanted = args.variants.split(',')
    for kind in args.kinds.split(','):
        for name, extra in variants:
            if name not in wanted:
                continue
            env = dict(os.environ)
            cache_dir = None
            if 'AMD_COMGR_CACHE_DIR' in extra:
                cache_dir = os.path.join(args.cache_root, kind)
                shutil.rmtree(cache_dir, ignore_errors=True)
                os.makedirs(cache_dir)
                extra = dict(extra, AMD_COMGR_CACHE_DIR=cache_dir)
            env.update(extra)
            for i in range(args.repeat):
                out = subprocess.run(
                    [sys.executable, os.path.abspath(__file__), '--child',
                     kind], env=env, stdout=subprocess.PIPE, timeout=120,
                    check=True)
                row = json.loads(out.stdout.decode().strip().splitlines()[-1])
                row.update(kind=kind, variant=name, run=i, gap_s=args.gap)
                time.sleep(args.gap)
                if cache_dir:
                    row['cache_files'] = cache_files(cache_dir)
                print(json.dumps(row), flush=True)
    print(json.dumps({'home_comgr_cache_after': os.path.isdir(home_cache),
                      'files': cache_files(home_cache)}), flush=True)
    return 0


if __name__ == '__main__':
    sys.exit(main())
