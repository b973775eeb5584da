"""Reconcile core, mirroring ``autoscaler/autoscaler_test.py`` case by case
(k8s fakes -> an actuator fake with the same string-typed fields) and adding
the gaps SURVEY §4 lists (processing-key counting, decision assertions)."""
import random

import pytest

import kiosk_autoscaler_amd as autoscaler
from kiosk_autoscaler_amd.gpumgr.resources import (ActuatorError, Metadata,
                                                   ResourceList, ResourceView,
                                                   Spec, Status)


def actuator_error(*_, **__):
    raise ActuatorError(500, 'thrown on purpose')


class DummyActuator(object):
    """String-typed counts exercise the int() cast, like DummyKubernetes."""

    def __init__(self):
        self.patches = []

    def list_namespaced_deployment(self, *_, **__):
        return ResourceList(items=[
            ResourceView(kind='deployment', metadata=Metadata(name='pod1'),
                         spec=Spec(replicas='4'),
                         status=Status(available_replicas=None)),
            ResourceView(kind='deployment', metadata=Metadata(name='pod2'),
                         spec=Spec(replicas='8'),
                         status=Status(available_replicas='8')),
        ])

    def list_namespaced_job(self, *_, **__):
        return ResourceList(items=[
            ResourceView(kind='job', metadata=Metadata(name='pod1'),
                         spec=Spec(completions='1', parallelism='1'),
                         status=Status()),
            ResourceView(kind='job', metadata=Metadata(name='pod2'),
                         spec=Spec(completions='2', parallelism='2'),
                         status=Status()),
        ])

    def patch_namespaced_deployment(self, name, namespace, body):
        self.patches.append(('deployment', name, namespace, body))
        return body

    def patch_namespaced_job(self, name, namespace, body):
        self.patches.append(('job', name, namespace, body))
        return body


def make(redis_client, queues='queue', **kw):
    return autoscaler.Autoscaler(redis_client, queues, actuator=DummyActuator(),
                                 **kw)


def test_package_surface():
    assert hasattr(autoscaler, 'redis')
    assert hasattr(autoscaler.redis, 'RedisClient')
    scaler = autoscaler.Autoscaler(None)
    assert scaler.redis_keys == {'predict': 0}      # ctor default queue
    assert scaler.managed_resource_types == {'deployment', 'job'}


def test_get_desired_pods(redis_client):
    scaler = make(redis_client)
    scaler.redis_keys['queue'] = 10
    assert scaler.get_desired_pods('queue', 2, 0, 2, 1) == 2    # > max
    assert scaler.get_desired_pods('queue', 5, 9, 10, 0) == 9   # < min
    assert scaler.get_desired_pods('queue', 3, 0, 5, 1) == 3    # in range
    assert scaler.get_desired_pods('queue', 10, 0, 5, 3) == 3   # hold current


@pytest.mark.parametrize('method,args', [
    ('list_namespaced_deployment', ('ns',)),
    ('list_namespaced_job', ('ns',)),
    ('patch_namespaced_deployment', ('pod', 'ns', {'spec': {'replicas': 1}})),
    ('patch_namespaced_job', ('job', 'ns', {'spec': {'parallelism': 1}})),
])
def test_actuator_wrappers_reraise(redis_client, method, args):
    scaler = make(redis_client)
    getattr(scaler, method)(*args)          # success path
    setattr(scaler.actuator, method, actuator_error)
    with pytest.raises(ActuatorError):
        getattr(scaler, method)(*args)


def test_get_current_pods(redis_client):
    scaler = make(redis_client)
    with pytest.raises(ValueError):
        scaler.get_current_pods('namespace', 'bad_type', 'pod')
    assert scaler.get_current_pods('ns', 'deployment', 'pod1') == 4
    assert scaler.get_current_pods('ns', 'deployment', 'pod2') == 8
    assert scaler.get_current_pods('ns', 'deployment', 'pod2', True) == 8
    assert scaler.get_current_pods('ns', 'deployment', 'pod1', True) == 0
    assert scaler.get_current_pods('ns', 'job', 'pod1') == 1
    assert scaler.get_current_pods('ns', 'job', 'pod2') == 2
    assert scaler.get_current_pods('ns', 'deployment', 'missing') == 0


def test_tally_queues(redis_client):
    expected = random.randint(1, 10)
    for _ in range(expected):
        redis_client.lpush('queue', 'jobHash')
    scaler = make(redis_client, queues='queue')
    scaler.tally_queues()
    assert scaler.redis_keys == {'queue': expected}

    queues = 'predict,track,train'
    expected = random.randint(1, 10)
    for q in queues.split(','):
        for _ in range(expected):
            redis_client.lpush(q, 'jobHash')
    scaler = make(redis_client, queues=queues)
    scaler.tally_queues()
    assert scaler.redis_keys == {q: expected for q in queues.split(',')}


def test_tally_counts_processing_keys(redis_client):
    """Characterised example from SURVEY §2.1 C6."""
    redis_client.rpush('predict', 'a', 'b')
    redis_client.rpush('processing-predict:h1', 'x', 'y', 'z')
    redis_client.rpush('processing-predict:h2', 'x')
    redis_client.rpush('processing-track', 'x')     # no colon: not matched
    scaler = make(redis_client, queues='predict,track')
    scaler.tally_queues()
    assert scaler.redis_keys == {'predict': 4, 'track': 0}
    assert scaler.in_progress == {'predict': 2, 'track': 0}


def test_scale_resource(redis_client):
    scaler = make(redis_client)
    assert not scaler.scale_resource(1, 1, 'deployment', 'ns', 'name')
    assert scaler.scale_resource(2, 1, 'job', 'ns', 'name')
    assert scaler.scale_resource(2, 1, 'deployment', 'ns', 'name')
    assert scaler.actuator.patches == [
        ('job', 'name', 'ns', {'spec': {'parallelism': 2}}),
        ('deployment', 'name', 'ns', {'spec': {'replicas': 2}})]
    with pytest.raises(ValueError):
        scaler.scale_resource(2, 1, 'badvalue', 'ns', 'name')


def test_scale(redis_client):
    scaler = make(redis_client, queues='predict,track')
    for resource_type in scaler.managed_resource_types:
        scaler.scale(namespace='namespace', resource_type=resource_type,
                     name='test')

    def bad_scale_resource(*args, **kwargs):
        raise ActuatorError(500, 'thrown on purpose')
    scaler.scale_resource = bad_scale_resource
    for resource_type in scaler.managed_resource_types:
        scaler.scale(namespace='namespace', resource_type=resource_type,
                     name='test')


def test_tick_event_is_stamped_at_the_decision_and_sent_after_the_patch(
        redis_client):
    """The ``tick`` event carries the decision instant but is sent once the
    actuator call returned (a Redis event sink's round trip stays off the
    PATCH), also when the PATCH fails."""
    from kiosk_autoscaler_amd.utils.events import EventLog
    events = EventLog(source='test')
    events.keep = True
    scaler = make(redis_client, events=events)
    redis_client.lpush('queue', 'a', 'b')
    sent = []
    actuator = scaler.actuator
    real = actuator.patch_namespaced_job

    def patch(*args):
        sent.append([e['ev'] for e in events.records])
        return real(*args)
    actuator.patch_namespaced_job = patch
    scaler.scale(namespace='ns', resource_type='job', name='pod1',
                 max_pods=4)
    assert sent == [[]]                     # nothing sent before the PATCH
    kinds = [e['ev'] for e in events.records]
    assert kinds == ['scale', 'tick']
    scale_ev, tick_ev = events.records
    assert tick_ev['t'] <= scale_ev['t'] and tick_ev['desired'] == 2
    actuator.patch_namespaced_job = actuator_error
    redis_client.lpush('queue', 'c')
    scaler.scale(namespace='ns', resource_type='job', name='pod1',
                 max_pods=4)
    assert events.records[-1]['ev'] == 'tick'


def test_scale_decisions(redis_client):
    """The reference test is smoke-only; assert the actual decisions."""
    scaler = make(redis_client, queues='predict,track')
    # pod1: 4 declared replicas; one key in each queue -> inflation to 8
    redis_client.lpush('predict', 'a')
    redis_client.lpush('track', 'b')
    assert scaler.scale('ns', 'deployment', 'pod1', 0, 8, 1) == 8
    assert scaler.actuator.patches[-1][3] == {'spec': {'replicas': 8}}
    redis_client.delete('predict', 'track')
    assert scaler.scale('ns', 'deployment', 'pod1', 0, 8, 1) == 0


def test_scale_tally_errors_propagate(redis_client):
    scaler = make(redis_client)
    redis_client.engine.inject_fault('LLEN', 'error')
    with pytest.raises(Exception):
        scaler.scale('ns', 'deployment', 'pod1')


def test_strict_policy_with_hysteresis(redis_client):
    clock = [0.0]
    scaler = make(redis_client, queues='predict', policy='strict',
                  scale_down_delay=10.0, clock=lambda: clock[0])
    scaler.actuator.list_namespaced_deployment = lambda ns: ResourceList(
        items=[ResourceView(kind='deployment', metadata=Metadata(name='w'),
                            spec=Spec(replicas=4),
                            status=Status(available_replicas=4))])
    redis_client.rpush('predict', 'a')
    assert scaler.scale('ns', 'deployment', 'w', 0, 8, 1) == 4  # held
    clock[0] = 11.0
    assert scaler.scale('ns', 'deployment', 'w', 0, 8, 1) == 1  # applied


def test_strict_default_holds_only_the_last_worker(redis_client):
    """Plain ``strict``: a scale-down that keeps
    workers applies at once; a target of zero keeps one worker until it
    was read on two ticks ``zero_delay`` apart -- an empty queue for one
    tick mid-burst does not make the next key pay a cold start."""
    clock = [0.0]
    replicas = [4]
    scaler = make(redis_client, queues='predict', policy='strict',
                  zero_delay=5.0, clock=lambda: clock[0])
    scaler.actuator.list_namespaced_deployment = lambda ns: ResourceList(
        items=[ResourceView(kind='deployment', metadata=Metadata(name='w'),
                            spec=Spec(replicas=replicas[0]),
                            status=Status(available_replicas=replicas[0]))])
    redis_client.rpush('predict', 'a', 'b')
    assert scaler.scale('ns', 'deployment', 'w', 0, 8, 1) == 2   # at once
    replicas[0] = 2
    redis_client.delete('predict')
    clock[0] = 5.0
    assert scaler.scale('ns', 'deployment', 'w', 0, 8, 1) == 1   # zero held
    replicas[0] = 1
    clock[0] = 7.0
    redis_client.rpush('predict', 'c')                           # a new key
    assert scaler.scale('ns', 'deployment', 'w', 0, 8, 1) == 1
    redis_client.delete('predict')
    clock[0] = 12.0
    assert scaler.scale('ns', 'deployment', 'w', 0, 8, 1) == 1   # held anew
    clock[0] = 17.0
    assert scaler.scale('ns', 'deployment', 'w', 0, 8, 1) == 0   # two ticks


@pytest.mark.parametrize('tally', ['reference', 'atomic'])
def test_strict_busy_floor_counts_workers_not_keys(redis_client, tally):
    """A batched (job) worker holds one processing key per slot: the strict
    floor is the number of busy *workers* (ADVICE r1 low), 1 here, not 4."""
    scaler = make(redis_client, queues='predict,track', policy='strict',
                  tally=tally)
    scaler.actuator.list_namespaced_job = lambda ns: ResourceList(
        items=[ResourceView(kind='job', metadata=Metadata(name='w'),
                            spec=Spec(parallelism=3),
                            status=Status(available_replicas=3))])
    for suffix in ('', '.1', '.2'):
        redis_client.rpush('processing-predict:w-g0-ab-1' + suffix, 'k')
    redis_client.rpush('processing-track:w-g0-ab-1.3', 'k')
    scaler.tally_queues()
    assert scaler.in_progress == {'predict': 3, 'track': 1}
    assert scaler.busy_workers == {'w-g0-ab-1'}
    # 4 keys, kpp 4 -> ceil 1; the floor is one busy worker, not 4 keys
    assert scaler.scale('ns', 'job', 'w', 0, 8, 4) == 1


def test_atomic_tally_matches_and_is_consistent(redis_client):
    """TALLY_MODE=atomic: LLEN + KEYS in one MULTI/EXEC.  A consumer that
    keeps moving items between the queue and processing keys never makes
    the atomic tally over- or under-count (SURVEY §5.2 race)."""
    import threading
    for i in range(20):
        redis_client.lpush('q', 'item%d' % i)
    from kiosk_autoscaler_amd import Autoscaler
    scaler = Autoscaler(redis_client, 'q', tally='atomic')
    assert scaler.tally_queues() == {'q': 20}
    stop = threading.Event()

    def churn():
        n = 0
        while not stop.is_set():
            key = 'processing-q:w%d' % (n % 7)
            if redis_client.lmove('q', key, 'RIGHT', 'LEFT') is None:
                continue
            # every move is atomic: the item is always in exactly one list
            redis_client.lmove(key, 'q', 'RIGHT', 'LEFT')
            n += 1
    thread = threading.Thread(target=churn, daemon=True)
    thread.start()
    try:
        for _ in range(200):
            assert scaler.tally_queues()['q'] == 20
    finally:
        stop.set()
        thread.join(5)
    with pytest.raises(ValueError):
        Autoscaler(redis_client, 'q', tally='nope')


def test_atomic_tally_through_sentinel_proxy_and_kredis(resp_server,
                                                         kredis_server):
    """The MULTI/EXEC tally over real sockets: the retrying proxy routes the
    pipeline to the master; both RESP servers implement MULTI + KEYS."""
    from kiosk_autoscaler_amd import Autoscaler
    from kiosk_autoscaler_amd.redisq import RedisClient
    for server in (resp_server, kredis_server):
        proxy = RedisClient(host=server.host, port=server.port, backoff=0)
        proxy.delete('q')
        proxy.lpush('q', 'a', 'b', 'c')
        proxy.lpush('processing-q:w1', 'x')
        proxy.lpush('processing-q:w2', 'y')
        proxy.lpush('processing-qq:w3', 'z')          # another queue
        scaler = Autoscaler(proxy, 'q', tally='atomic')
        assert scaler.tally_queues() == {'q': 5}
        assert scaler.in_progress == {'q': 2}
