#!/usr/bin/env python3
"""Control-plane cost of one reconcile tick (``Autoscaler.scale``).

BASELINE.md §3 quotes the reference's per-tick overhead as 0.61 ms/tick
(its Python classes with stub Redis/Kubernetes, 2 queues, a 1 010-key
keyspace).  This measures the same tick here in three setups:

* ``inproc``  -- in-process fake Redis + an in-memory actuator (the
  reference measurement's shape: no sockets);
* ``kredis``  -- the native RESP server over loopback TCP + the in-memory
  actuator (what a real tick pays for its Redis round trips);
* ``manager`` -- ``kredis`` plus the real embedded GPU manager as the
  actuator (mock CPU backend, no workers spawned: MAX_PODS = 0 keeps the
  decision at 0).

Both tally modes (``reference`` = LLEN + SCAN, ``atomic`` = one MULTI/EXEC)
are reported.  Logging is silenced, as the reference measurement's was not
dominated by it.

    python tools/bench_tick.py [--ticks 2000] [--modes inproc,kredis,manager]
"""
import argparse
import json
import logging
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kiosk_autoscaler_amd import Autoscaler  # noqa: E402
from kiosk_autoscaler_amd.gpumgr.resources import (  # noqa: E402
    Metadata, ResourceList, ResourceView, Spec, Status)

QUEUES = 'predict,track'


class MemoryActuator(object):
    """One deployment, declared 0 replicas; records PATCHes."""

    def __init__(self):
        self.replicas = 0
        self.patches = 0

    def list_namespaced_deployment(self, *_):
        return ResourceList(items=[ResourceView(
            kind='deployment', metadata=Metadata(name='bench'),
            spec=Spec(replicas=self.replicas),
            status=Status(available_replicas=self.replicas))])

    def list_namespaced_job(self, *_):
        return ResourceList(items=[])

    def patch_namespaced_deployment(self, name, namespace, body):
        self.patches += 1
        self.replicas = body['spec']['replicas']
        return body

    patch_namespaced_job = patch_namespaced_deployment


def populate(redis):
    """2 queues with items, 8 processing keys, job hashes: 1 010 keys."""
    pipe = redis.pipeline(transaction=False)
    for i in range(5):
        pipe.rpush('predict', 'job-%d' % i)
        pipe.rpush('track', 'job-t%d' % i)
    for i in range(4):
        pipe.rpush('processing-predict:w%d' % i, 'job-p%d' % i)
        pipe.rpush('processing-track:w%d' % i, 'job-q%d' % i)
    for i in range(1010 - 2 - 8):
        pipe.hset('job-%d' % i, mapping={'status': 'new', 'rows': '2048'})
    pipe.execute()


def free_port():
    sock = socket.socket()
    sock.bind(('127.0.0.1', 0))
    port = sock.getsockname()[1]
    sock.close()
    return port


def time_ticks(scaler, ticks, max_pods):
    for _ in range(20):
        scaler.scale('bench', 'deployment', 'bench', 0, max_pods, 1)
    samples = []
    for _ in range(ticks):
        t0 = time.perf_counter()
        scaler.scale('bench', 'deployment', 'bench', 0, max_pods, 1)
        samples.append((time.perf_counter() - t0) * 1e3)
    samples.sort()
    return {'ticks': ticks,
            'mean_ms': round(sum(samples) / len(samples), 4),
            'p50_ms': round(samples[len(samples) // 2], 4),
            'p99_ms': round(samples[int(len(samples) * 0.99)], 4)}


def run_mode(mode, ticks):
    from kiosk_autoscaler_amd.redisq import StrictRedis
    out = []
    server = None
    manager = None
    try:
        if mode == 'inproc':
            from kiosk_autoscaler_amd.fakes import FakeRedis, RedisEngine
            redis = FakeRedis(engine=RedisEngine(), decode_responses=True)
        else:
            binary = os.path.join(ROOT, 'build', 'kredis-server')
            if not os.path.exists(binary):
                raise RuntimeError('kredis-server not built '
                                   '(python tools/build_native.py)')
            port = free_port()
            server = subprocess.Popen([binary, '--port', str(port)],
                                      stdout=subprocess.DEVNULL,
                                      stderr=subprocess.DEVNULL)
            redis = StrictRedis(host='127.0.0.1', port=port,
                                decode_responses=True)
            deadline = time.time() + 10
            while True:
                try:
                    if redis.ping():
                        break
                except Exception:  # pylint: disable=broad-except
                    if time.time() > deadline:
                        raise
                    time.sleep(0.02)
        populate(redis)
        if mode == 'manager':
            from kiosk_autoscaler_amd.gpumgr.controller import (
                GpuManager, WorkerTemplate)
            from kiosk_autoscaler_amd.gpumgr.gpus import GpuSlot
            manager = GpuManager([GpuSlot(0, '', kind='cpu')], pool_size=0)
            manager.register('deployment', 'bench', 'bench',
                             WorkerTemplate(queues=QUEUES.split(','),
                                            backend='cpu'))
            manager.start()
            actuator = manager
            max_pods = 0
        else:
            actuator = MemoryActuator()
            max_pods = 0
        for tally in ('reference', 'atomic'):
            scaler = Autoscaler(redis, QUEUES, actuator=actuator,
                                tally=tally)
            row = {'mode': mode, 'tally': tally, 'queues': QUEUES,
                   'keyspace': 1010}
            row.update(time_ticks(scaler, ticks, max_pods))
            out.append(row)
    finally:
        if manager is not None:
            manager.stop()
        if server is not None:
            server.terminate()
            server.wait(timeout=10)
    return out


def main():
    parser = argparse.ArgumentParser()
    parser.add_argument('--ticks', type=int, default=2000)
    parser.add_argument('--modes', default='inproc,kredis,manager')
    args = parser.parse_args()
    logging.disable(logging.CRITICAL)
    for mode in args.modes.split(','):
        for row in run_mode(mode, args.ticks):
            row['reference_ms_per_tick'] = 0.61
            print(json.dumps(row), flush=True)


if __name__ == '__main__':
    main()
