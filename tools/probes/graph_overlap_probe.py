#!/usr/bin/env python3
"""Can a standby pay the runtime's first graph instantiation off its
critical path?

ROCm 7.2's first ``hipGraphInstantiate`` in a process costs 14-16 ms
(``profiles/r4_comgr/first_graph.jsonl``), paid inside every standby's
engine build.  Each child (a fresh process on ``/opt/rocm``'s runtime)
opens the context, then in one of these orders:

* ``serial``: first stream, then a one-memset graph (instantiate, launch);
* ``graph_first``: the graph (built with ``hipGraphAddMemsetNode``, no
  stream) before the first stream;
* ``overlap``: the graph on a second thread while the main thread creates
  the first stream;
* ``empty_first``: an empty-node graph first: does it pay the one-time
  cost for the memset graph after it?

It prints ms per step and the wall from the context to a launched graph.

    python tools/graph_overlap_probe.py --repeat 3
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import threading
import time


class MemsetParams(ctypes.Structure):
    _fields_ = [('dst', ctypes.c_void_p), ('elementSize', ctypes.c_uint),
                ('height', ctypes.c_size_t), ('pitch', ctypes.c_size_t),
                ('value', ctypes.c_uint), ('width', ctypes.c_size_t)]


def child(mode):
    hip = ctypes.CDLL('/opt/rocm/lib/libamdhip64.so.7')
    row = {'mode': mode}
    t = [time.perf_counter()]

    def mark(name):
        now = time.perf_counter()
        row[name] = round((now - t[0]) * 1e3, 2)
        t[0] = now
    start = time.perf_counter()
    hip.hipFree(ctypes.c_void_p(0))
    mark('context')
    after_ctx = time.perf_counter()
    buf = ctypes.c_void_p()
    hip.hipMalloc(ctypes.byref(buf), ctypes.c_size_t(4096))
    stream = ctypes.c_void_p()
    exe = ctypes.c_void_p()

    def memset_graph(out):
        graph, node = ctypes.c_void_p(), ctypes.c_void_p()
        params = MemsetParams(buf, 4, 1, 0, 0, 1024)
        g0 = time.perf_counter()
        hip.hipGraphCreate(ctypes.byref(graph), 0)
        hip.hipGraphAddMemsetNode(ctypes.byref(node), graph, None,
                                  ctypes.c_size_t(0), ctypes.byref(params))
        rc = hip.hipGraphInstantiate(ctypes.byref(out), graph, None, None,
                                     ctypes.c_size_t(0))
        row['graph_thread_ms'] = round((time.perf_counter() - g0) * 1e3, 2)
        row['graph_rc'] = rc

    def empty_graph():
        graph, node, ex = ctypes.c_void_p(), ctypes.c_void_p(), \
            ctypes.c_void_p()
        hip.hipGraphCreate(ctypes.byref(graph), 0)
        hip.hipGraphAddEmptyNode(ctypes.byref(node), graph, None,
                                 ctypes.c_size_t(0))
        hip.hipGraphInstantiate(ctypes.byref(ex), graph, None, None,
                                ctypes.c_size_t(0))

    if mode == 'serial':
        hip.hipStreamCreate(ctypes.byref(stream))
        mark('stream')
        memset_graph(exe)
        mark('graph')
    elif mode == 'graph_first':
        memset_graph(exe)
        mark('graph')
        hip.hipStreamCreate(ctypes.byref(stream))
        mark('stream')
    elif mode == 'overlap':
        th = threading.Thread(target=memset_graph, args=(exe,))
        th.start()
        hip.hipStreamCreate(ctypes.byref(stream))
        mark('stream')
        th.join()
        mark('graph_join')
    elif mode == 'empty_first':
        empty_graph()
        mark('empty_graph')
        hip.hipStreamCreate(ctypes.byref(stream))
        mark('stream')
        memset_graph(exe)
        mark('graph')
    rc = hip.hipGraphLaunch(exe, stream)
    hip.hipStreamSynchronize(stream)
    mark('launch')
    row['launch_rc'] = rc
    row['after_context_ms'] = round((time.perf_counter() - after_ctx) * 1e3,
                                    2)
    row['total_ms'] = round((time.perf_counter() - start) * 1e3, 2)
    print(json.dumps(row), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--child')
    ap.add_argument('--repeat', type=int, default=3)
    args = ap.parse_args()
    if args.child:
        child(args.child)
        return 0
    modes = ['serial', 'graph_first', 'overlap', 'empty_first']
    # one throw-away child fills comgr's cache (profiles/r4_comgr)
    for rnd in range(args.repeat + 1):
        for mode in modes:
            out = subprocess.run([sys.executable, '-S', os.path.abspath(
                __file__), '--child', mode], stdout=subprocess.PIPE,
                timeout=60, check=True)
            if rnd:
                sys.stdout.write(out.stdout.decode())
                sys.stdout.flush()
    return 0


if __name__ == '__main__':
    sys.exit(main())
