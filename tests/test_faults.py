"""Fault injection and failure detection: a crashed, hung,
slow-starting or failing worker is detected (waitpid / watchdog), its
in-flight item requeued and a replacement serves it; a dropped Redis socket
is survived transparently.  CPU mock workers over a real RESP socket."""
import pytest

from kiosk_autoscaler_amd.fakes import FakeRedis
from kiosk_autoscaler_amd.utils import faults
from test_integration_cpu import enqueue, stack, tick, wait_for  # noqa: F401


def test_parse_spec():
    assert faults.parse('') == {}
    assert faults.parse('hang_key=2:500, fail_start') == {
        'hang_key': (2.0, 500.0), 'fail_start': ()}
    assert faults.parse('crash_key=3') == {'crash_key': (3.0,)}
    for bad in ('explode=1', 'crash_key', 'slow_start'):
        with pytest.raises(ValueError):
            faults.parse(bad)


def test_fault_fires_once_across_workers():
    redis = FakeRedis()
    first = faults.FaultPlan(faults.parse('fail_start'), redis, owner='w-1')
    second = faults.FaultPlan(faults.parse('fail_start'), redis, owner='w-2')
    with pytest.raises(faults.InjectedFault):
        first.at_start()
    second.at_start()                       # already claimed by w-1
    first.at_start()                        # and never twice in one process
    assert redis.get('kiosk:fault:fail_start') == 'w-1'
    local = faults.FaultPlan(faults.parse('hang_key=2:1'))
    local.before_key(1)
    assert local.fired == []
    local.before_key(2)
    assert local.fired == ['hang_key']


def _served_once_after_failure(s, client, manager, scaler, events):
    enqueue(client, 1)
    assert tick(scaler, s) == 1
    wait_for(lambda: client.hget('predict:job0', 'status') == 'done',
             timeout=40)
    history = manager.history
    assert history and history[0]['exit_code'] != 0
    view = manager.list_namespaced_deployment('default').items[0]
    assert view.status.restarts >= 1
    return history[0]


@pytest.mark.slow
def test_hung_worker_killed_by_watchdog(stack):
    s, client, manager, scaler, events = stack(
        extra_env={'KIOSK_FAULTS': 'hang_key=1:60000'}, WARM_POOL='0',
        WORKER_TIMEOUT='1.0')
    dead = _served_once_after_failure(s, client, manager, scaler, events)
    assert dead['killed'].startswith('no progress')
    kinds = [e['ev'] for e in events.records]
    assert 'worker_timeout' in kinds and 'requeue' in kinds


@pytest.mark.slow
def test_crash_mid_key_requeues(stack):
    s, client, manager, scaler, events = stack(
        extra_env={'KIOSK_FAULTS': 'crash_key=1'}, WARM_POOL='0')
    dead = _served_once_after_failure(s, client, manager, scaler, events)
    assert dead['exit_code'] == faults.CRASH_CODE and not dead['killed']
    assert any(e['ev'] == 'requeue' for e in events.records)


@pytest.mark.slow
def test_start_failure_and_start_timeout(stack):
    s, client, manager, scaler, events = stack(
        extra_env={'KIOSK_FAULTS': 'fail_start'}, WARM_POOL='0')
    dead = _served_once_after_failure(s, client, manager, scaler, events)
    assert dead['exit_code'] == 3 and dead['t_ready'] is None


@pytest.mark.slow
def test_slow_start_killed_by_start_timeout(stack):
    s, client, manager, scaler, events = stack(
        extra_env={'KIOSK_FAULTS': 'slow_start=60000'}, WARM_POOL='1',
        WORKER_TIMEOUT='2.0:2.0')       # busy bound : start bound
    dead = _served_once_after_failure(s, client, manager, scaler, events)
    assert dead['killed'].startswith('not READY')


@pytest.mark.slow
def test_dropped_redis_socket_is_survived(stack):
    s, client, manager, scaler, events = stack(
        extra_env={'KIOSK_FAULTS': 'drop_redis_key=1'}, WARM_POOL='0')
    enqueue(client, 2)
    assert tick(scaler, s) == 1
    wait_for(lambda: all(client.hget('predict:job%d' % i, 'status') == 'done'
                         for i in range(2)), timeout=30)
    assert manager.history == []        # nobody died
    assert client.get('kiosk:fault:drop_redis_key')


@pytest.mark.gpu
def test_gpu_hung_kernel_killed_by_watchdog(stack):
    """A real stuck GPU job: the worker's serving stream runs the bounded
    spin kernel; the watchdog SIGKILLs the process mid-kernel, the item is
    requeued and a fresh HIP worker on the same GPU serves it."""
    s, client, manager, scaler, events = stack(
        extra_env={'KIOSK_FAULTS': 'hang_key=1:20000'}, WARM_POOL='1',
        WORKER_BACKEND='hip', WORKER_TIMEOUT='2.0', FENCE='none',
        MODEL='1024x4096x2',
        ROWS_PER_KEY='256')
    wait_for(lambda: manager.standbys and all(
        p.booted for p in manager.standbys.values()), timeout=120)
    enqueue(client, 1)
    assert tick(scaler, s) == 1
    wait_for(lambda: client.hget('predict:job0', 'status') == 'done',
             timeout=120)
    dead = manager.history[0]
    assert dead['killed'].startswith('no progress')
    assert float(client.hget('predict:job0', 'compute_ms')) > 0


@pytest.mark.gpu
def test_gpu_worker_recycled_and_reused(stack):
    """A drained HIP worker frees its engine and becomes the GPU's standby;
    the next scale-up on that GPU reuses the same process (HIP context kept)
    and serves with a freshly built engine."""
    s, client, manager, scaler, events = stack(
        WARM_POOL='1', WORKER_BACKEND='hip', FENCE='none',
        MODEL='1024x4096x2',
        ROWS_PER_KEY='256')
    wait_for(lambda: manager.standbys and all(
        p.booted for p in manager.standbys.values()), timeout=120)
    pid = manager.standbys[0].pid
    for round_ in range(2):
        client.delete('predict:job0')
        enqueue(client, 1)
        assert tick(scaler, s) == 1
        wait_for(lambda: client.hget('predict:job0', 'status') == 'done',
                 timeout=120)
        worker = manager.status()['resources'][0]['workers'][0]
        assert worker['pid'] == pid and worker['from_pool']
        assert tick(scaler, s) == 0
        wait_for(lambda: 0 in manager.standbys and
                 manager.standbys[0].booted, timeout=60)
        assert manager.standbys[0].pid == pid
    ready = [e for e in events.records if e['ev'] == 'worker_recycled']
    assert len(ready) == 2
