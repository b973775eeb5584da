"""GPUMGR=k8s: the reconcile core driving the Kubernetes API, as the
reference does.  The ``kubernetes`` package is replaced by an in-process
fake module (the reference's own strategy: ``DummyKubernetes`` patched in
for ``AppsV1Api``/``BatchV1Api``, ``autoscaler/autoscaler_test.py:54-81``);
counts are strings to exercise the ``int()`` cast."""
import sys
import types

import pytest

from kiosk_autoscaler_amd import Autoscaler, gpumgr
from kiosk_autoscaler_amd.fakes import FakeRedis
from kiosk_autoscaler_amd.gpumgr.resources import ActuatorError


class Bunch(object):
    def __init__(self, **kw):
        self.__dict__.update(kw)


class ApiException(Exception):
    def __init__(self, status=500, reason='boom'):
        Exception.__init__(self, reason)
        self.status = status
        self.reason = reason
        self.body = None


class FakeApi(object):
    patches = []
    fail_patch = False

    def list_namespaced_deployment(self, namespace):
        return Bunch(items=[Bunch(
            metadata=Bunch(name='worker'),
            spec=Bunch(replicas='2'),
            status=Bunch(available_replicas='1'))])

    def list_namespaced_job(self, namespace):
        return Bunch(items=[Bunch(metadata=Bunch(name='jobworker'),
                                  spec=Bunch(parallelism='1'),
                                  status=Bunch())])

    def patch_namespaced_deployment(self, name, namespace, body):
        if FakeApi.fail_patch:
            raise ApiException(409, 'conflict')
        FakeApi.patches.append(('deployment', name, namespace, body))
        return body

    def patch_namespaced_job(self, name, namespace, body):
        FakeApi.patches.append(('job', name, namespace, body))
        return body


@pytest.fixture
def fake_kubernetes(monkeypatch):
    mod = types.ModuleType('kubernetes')
    client = types.ModuleType('kubernetes.client')
    config = types.ModuleType('kubernetes.config')
    rest = types.ModuleType('kubernetes.client.rest')
    rest.ApiException = ApiException
    client.rest = rest
    client.AppsV1Api = FakeApi
    client.BatchV1Api = FakeApi
    loaded = []
    config.load_incluster_config = lambda: loaded.append('incluster')
    config.load_kube_config = lambda: loaded.append('kubeconfig')
    mod.client = client
    mod.config = config
    for name, m in (('kubernetes', mod), ('kubernetes.client', client),
                    ('kubernetes.config', config),
                    ('kubernetes.client.rest', rest)):
        monkeypatch.setitem(sys.modules, name, m)
    FakeApi.patches = []
    FakeApi.fail_patch = False
    return loaded


def test_connect_k8s_and_scale(fake_kubernetes):
    actuator = gpumgr.connect('k8s')
    assert fake_kubernetes == ['incluster']
    redis = FakeRedis()
    for i in range(3):
        redis.lpush('predict', 'k%d' % i)
    scaler = Autoscaler(redis, 'predict', actuator=actuator)
    assert scaler.get_current_pods('ns', 'deployment', 'worker') == 2
    assert scaler.get_current_pods('ns', 'deployment', 'worker',
                                   only_running=True) == 1
    scaler.scale('ns', 'deployment', 'worker', min_pods=0, max_pods=4,
                 keys_per_pod=1)
    assert FakeApi.patches == [('deployment', 'worker', 'ns',
                                {'spec': {'replicas': 3}})]
    scaler.scale('ns', 'job', 'jobworker', min_pods=0, max_pods=4,
                 keys_per_pod=1)
    assert FakeApi.patches[-1] == ('job', 'jobworker', 'ns',
                                   {'spec': {'parallelism': 3}})
    gpumgr.connect('k8s-kubeconfig')
    assert fake_kubernetes[-1] == 'kubeconfig'


def test_api_exception_becomes_actuator_error(fake_kubernetes):
    actuator = gpumgr.connect('k8s')
    FakeApi.fail_patch = True
    with pytest.raises(ActuatorError) as info:
        actuator.patch_namespaced_deployment('worker', 'ns',
                                             {'spec': {'replicas': 1}})
    assert info.value.status == 409
    # the core swallows a failed PATCH (retried next tick), like the reference
    redis = FakeRedis()
    redis.lpush('predict', 'k')
    Autoscaler(redis, 'predict', actuator=actuator).scale(
        'ns', 'deployment', 'worker', 0, 4, 1)


def test_missing_package_is_a_clear_error(monkeypatch):
    monkeypatch.setitem(sys.modules, 'kubernetes', None)
    with pytest.raises(ActuatorError) as info:
        gpumgr.connect('k8s')
    assert info.value.status == 503 and 'kubernetes' in str(info.value)


def _standalone(resp_server, tmp_path, **env):
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    full = dict(os.environ, PYTHONPATH=root, REDIS_HOST=resp_server.host,
                REDIS_PORT=str(resp_server.port), QUEUES='predict',
                REDIS_INTERVAL='0', MOCK_WORK_MS='10')
    full.update(env)
    return subprocess.Popen(
        [sys.executable, '-m', 'kiosk_autoscaler_amd.worker.main',
         '--standalone', '--backend', 'cpu'], env=full, cwd=str(tmp_path),
        stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)


def _wait(pred, timeout=30):
    import time
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        if pred():
            return True
        time.sleep(0.05)
    raise AssertionError('timeout')


@pytest.mark.slow
def test_standalone_worker_pod_drains_on_sigterm(resp_server, tmp_path):
    """The worker as a plain Kubernetes pod (GPUMGR=k8s deployments):
    hostname-named processing keys, graceful exit 0 on SIGTERM."""
    import signal
    from kiosk_autoscaler_amd.redisq import StrictRedis
    client = StrictRedis(host=resp_server.host, port=resp_server.port,
                         decode_responses=True)
    proc = _standalone(resp_server, tmp_path, WORKER_ID='pod-a')
    try:
        for i in range(3):
            client.hset('predict:k%d' % i, mapping={'status': 'new'})
            client.lpush('predict', 'predict:k%d' % i)
        _wait(lambda: all(client.hget('predict:k%d' % i, 'status') == 'done'
                          for i in range(3)))
        assert client.hget('predict:k0', 'worker') == 'pod-a'
        proc.send_signal(signal.SIGTERM)
        assert proc.wait(20) == 0
        assert not list(client.scan_iter(match='processing-predict:*'))
    finally:
        if proc.poll() is None:
            proc.kill()


@pytest.mark.slow
def test_standalone_job_pod_completes(resp_server, tmp_path):
    from kiosk_autoscaler_amd.redisq import StrictRedis
    client = StrictRedis(host=resp_server.host, port=resp_server.port,
                         decode_responses=True)
    client.lpush('predict', 'plain-item')
    proc = _standalone(resp_server, tmp_path, WORKER_ID='job-a',
                       RESOURCE_TYPE='job', JOB_IDLE_EXIT_S='0.3')
    assert proc.wait(30) == 0          # the Job's pod completes
    assert client.llen('predict') == 0
