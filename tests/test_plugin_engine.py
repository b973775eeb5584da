"""``WORKER_ENGINE`` plug-in engines (models/plugin.py): the reference
scales whatever consumer its Deployment runs, so a user must be able to
bring a model and keep the rest of the worker (queue protocol, batching,
poison-job handling, standby pool, recycling).  Unit level on the runtime
with the in-proc fake Redis; integration level through the manager with
mock CPU workers; the PyTorch example on MI355X (``-m gpu``)."""
import os
import time

import pytest

from kiosk_autoscaler_amd.models import plugin
from kiosk_autoscaler_amd.worker import runtime as rt

REVERSE = 'kiosk_autoscaler_amd.models.plugin:ReverseEngine'


class _Channel(object):
    def __init__(self):
        self.events = []
        self.direct = {}

    def emit(self, ev, **fields):
        self.events.append((ev, fields))


def _runtime(redis_client, spec=REVERSE, batch=1, kind='deployment'):
    env = {'ROWS_PER_KEY': '64', 'WORKER_BATCH': str(batch),
           'QUEUES': 'predict'}
    cfg = rt.WorkerConfig(env, {'worker_id': 'w-g0-p-1', 'kind': kind})
    run = rt.WorkerRuntime(cfg, None, _Channel(), lambda: redis_client)
    run.redis = redis_client
    run.engine = plugin.PluginEngine(spec, cfg)
    run.engine.warmstart()
    return run


def _push(client, name, **fields):
    client.hset(name, mapping=dict({'status': 'new'}, **fields))
    client.lpush('predict', name)


def test_load_factory_contract():
    assert plugin.load_factory(REVERSE) is plugin.ReverseEngine
    with pytest.raises(ValueError, match='module:callable'):
        plugin.load_factory('no_colon_here')
    with pytest.raises(AttributeError):
        plugin.load_factory('kiosk_autoscaler_amd.models.plugin:Missing')
    with pytest.raises(TypeError, match='not callable'):
        plugin.load_factory('kiosk_autoscaler_amd.models.plugin:__doc__')


def test_engine_without_infer_is_refused():
    cfg = rt.WorkerConfig({}, {'worker_id': 'w'})
    with pytest.raises(TypeError, match='infer'):
        plugin.PluginEngine('kiosk_autoscaler_amd.models.mlp:CpuMlpEngine',
                            cfg)


def test_outputs_written_into_each_job_hash(redis_client):
    run = _runtime(redis_client, batch=3, kind='job')
    for i, text in enumerate(('abc', 'hello', 'xy')):
        _push(redis_client, 'predict:p%d' % i, payload=text)
    consumer = rt.QueueConsumer(redis_client, 'w-g0-p-1', ['predict'])
    run._process(consumer, consumer.pull(limit=3, block=False))
    got = {i: redis_client.hgetall('predict:p%d' % i) for i in range(3)}
    assert got[0]['output'] == 'rev:cba' and got[1]['output'] == 'rev:olleh'
    assert all(g['status'] == 'done' and g['worker'] == 'w-g0-p-1'
               and float(g['compute_ms']) >= 0 for g in got.values())
    assert run.keys_done == 3
    assert not list(redis_client.scan_iter(match='processing-predict:*'))


def test_rejected_batch_fails_and_worker_keeps_serving(redis_client):
    run = _runtime(redis_client)
    consumer = rt.QueueConsumer(redis_client, 'w-g0-p-1', ['predict'])
    _push(redis_client, 'predict:nopayload', rows=8)
    _push(redis_client, 'predict:ok', payload='ok')
    for _ in range(2):
        run._process(consumer, consumer.pull(limit=1, block=False))
    bad = redis_client.hgetall('predict:nopayload')
    assert bad['status'] == 'failed' and 'payload' in bad['reason']
    assert redis_client.hget('predict:ok', 'output') == 'rev:ko'
    assert not list(redis_client.scan_iter(match='processing-predict:*'))


def test_wrong_result_count_fails_the_batch(redis_client):
    run = _runtime(redis_client)
    run.engine.user.infer = lambda jobs: []
    consumer = rt.QueueConsumer(redis_client, 'w-g0-p-1', ['predict'])
    _push(redis_client, 'predict:z', payload='z')
    run._process(consumer, consumer.pull(limit=1, block=False))
    assert 'results for 1 jobs' in redis_client.hget('predict:z', 'reason')


def test_plugin_through_the_manager_with_recycling(resp_server):
    """Mock CPU workers running the plug-in: two scale 0 -> 1 -> 0 cycles;
    the second assignment finds the plug-in engine cached in the recycled
    standby (no second construction)."""
    from kiosk_autoscaler_amd import Autoscaler, gpumgr
    from kiosk_autoscaler_amd.config import Config, Settings
    from kiosk_autoscaler_amd.redisq import RedisClient, StrictRedis
    from kiosk_autoscaler_amd.utils.events import EventLog, drain_redis
    env = {'REDIS_HOST': resp_server.host, 'REDIS_PORT': str(resp_server.port),
           'QUEUES': 'predict', 'RESOURCE_NAME': 'plug', 'MAX_PODS': '1',
           'WORKER_BACKEND': 'cpu', 'WARM_POOL': '1', 'FENCE': 'none',
           'INTERVAL': '1', 'REDIS_INTERVAL': '0',
           'EVENT_LOG': 'redis',
           'POOL_IDLE_RELEASE_S': '0'}
    os.environ['WORKER_ENGINE'] = REVERSE
    try:
        s = Settings(Config(environ=env, use_files=False))
        client = StrictRedis(host=resp_server.host, port=resp_server.port,
                             decode_responses=True)
        events = EventLog(source='test', redis_client=client)
        manager = gpumgr.build_manager(s, redis_client=client,
                                       events=events).start()
    finally:
        del os.environ['WORKER_ENGINE']
    scaler = Autoscaler(RedisClient(host=resp_server.host,
                                    port=resp_server.port, backoff=0),
                        'predict', actuator=manager)

    def until(predicate, timeout=60):
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            if predicate():
                return
            time.sleep(0.02)
        raise AssertionError('timed out')
    try:
        for cycle, text in enumerate(('first', 'second')):
            item = 'predict:plug%d' % cycle
            client.hset(item, mapping={'status': 'new', 'payload': text})
            client.lpush('predict', item)
            assert scaler.scale('default', 'deployment', 'plug', 0, 1, 1) == 1
            # done is written before the processing key is DELeted
            until(lambda: client.hget(item, 'status') == 'done' and
                  not list(client.scan_iter(match='processing-*')))
            assert client.hget(item, 'output') == 'rev:' + text[::-1]
            assert scaler.scale('default', 'deployment', 'plug', 0, 1, 1) == 0
            until(lambda: not [w for r in manager.resources.values()
                               for w in r.workers.values()])
    finally:
        manager.stop(timeout=15)
    records = drain_redis(client)
    warm = [e for e in records if e['ev'] == 'warmstart']
    assert len(warm) == 2 and warm[0]['backend'] == 'cpu-example'
    # device-mode standbys build their engine at boot (round 4): both
    # assignments find it built
    assert [e['reused'] for e in warm] == [True, True]


@pytest.mark.gpu
def test_gpu_torch_engine_plugin_serves_on_mi355x(resp_server):
    """The PyTorch example engine as a plug-in on MI355X: the worker
    imports torch first (one HIP runtime), serves a job, and the written
    output matches an fp32 reference of the same model."""
    from kiosk_autoscaler_amd import gpumgr
    from kiosk_autoscaler_amd.config import Config, Settings
    from kiosk_autoscaler_amd.models.torch_engine import TorchMlpEngine
    from kiosk_autoscaler_amd.redisq import StrictRedis
    env = {'REDIS_HOST': resp_server.host, 'REDIS_PORT': str(resp_server.port),
           'QUEUES': 'predict', 'RESOURCE_NAME': 'torchplug',
           'MAX_PODS': '1', 'WORKER_BACKEND': 'hip', 'WARM_POOL': '0',
           'FENCE': 'none', 'REDIS_INTERVAL': '0', 'GPU_IDS': '0',
           'MODEL': '512x2048x2',
           'ROWS_PER_KEY': '64'}
    spec = 'kiosk_autoscaler_amd.models.torch_engine:TorchMlpEngine'
    os.environ['WORKER_ENGINE'] = spec
    try:
        s = Settings(Config(environ=env, use_files=False))
        client = StrictRedis(host=resp_server.host, port=resp_server.port,
                             decode_responses=True)
        manager = gpumgr.build_manager(s, redis_client=client).start()
    finally:
        del os.environ['WORKER_ENGINE']
    try:
        client.hset('predict:t0', mapping={'status': 'new', 'rows': 64,
                                           'seed': 7})
        client.lpush('predict', 'predict:t0')
        manager.patch_namespaced_deployment(
            'torchplug', 'default', {'spec': {'replicas': 1}})
        deadline = time.monotonic() + 180
        while client.hget('predict:t0', 'status') not in ('done', 'failed'):
            assert time.monotonic() < deadline, 'no result'
            time.sleep(0.05)
        fields = client.hgetall('predict:t0')
        assert fields['status'] == 'done', fields
        assert fields['engine'] == 'torch'
    finally:
        manager.stop(timeout=20)
    cfg = rt.WorkerConfig({'MODEL': '512x2048x2', 'ROWS_PER_KEY': '64'},
                          {'worker_id': 'ref'})
    ref = TorchMlpEngine(cfg).reference(64, 7)
    want = float(ref.sum())
    got = float(fields['output_sum'])
    scale = float(ref.abs().sum())
    assert abs(got - want) <= 2e-2 * scale, (got, want, scale)
