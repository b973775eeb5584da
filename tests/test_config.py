"""Env configuration surface."""
import pytest

from kiosk_autoscaler_amd.config import (Config, Settings, UndefinedValueError,
                                         cast_bool)


def test_reference_defaults(tmp_path):
    cfg = Config(environ={'RESOURCE_NAME': 'w'}, search_path=str(tmp_path))
    s = Settings(cfg)
    assert s.REDIS_HOST == 'redis-master'
    assert s.REDIS_PORT == 6379 and s.REDIS_INTERVAL == 1
    assert s.QUEUES == 'predict,track' and s.QUEUE_DELIMITER == ','
    assert s.INTERVAL == 5
    assert s.RESOURCE_NAMESPACE == 'default'
    assert s.RESOURCE_TYPE == 'deployment'
    assert (s.MIN_PODS, s.MAX_PODS, s.KEYS_PER_POD) == (0, 1, 1)
    assert s.queues == ['predict', 'track']
    assert s.SCALE_POLICY == 'reference'


def test_resource_name_required(tmp_path):
    cfg = Config(environ={}, search_path=str(tmp_path))
    with pytest.raises(UndefinedValueError):
        Settings(cfg)


def test_casts_and_env_precedence(tmp_path):
    (tmp_path / '.env').write_text('MAX_PODS=3\nQUEUES="a|b"\n'
                                   'export INTERVAL=2\n# comment\n')
    cfg = Config(environ={'RESOURCE_NAME': 'x', 'MAX_PODS': '8',
                          'QUEUE_DELIMITER': '|'},
                 search_path=str(tmp_path))
    s = Settings(cfg)
    assert s.MAX_PODS == 8          # env beats file
    assert s.INTERVAL == 2          # file beats default
    assert s.queues == ['a', 'b']
    assert cfg.source.endswith('.env')
    with pytest.raises(ValueError):
        Config(environ={'MAX_PODS': 'many'}, use_files=False)(
            'MAX_PODS', default=1, cast=int)


def test_settings_ini(tmp_path):
    (tmp_path / 'settings.ini').write_text('[settings]\nMIN_PODS=2\n')
    sub = tmp_path / 'a' / 'b'
    sub.mkdir(parents=True)
    s = Settings(Config(environ={'RESOURCE_NAME': 'n'}, search_path=str(sub)))
    assert s.MIN_PODS == 2


def test_cast_bool():
    assert cast_bool('yes') and cast_bool('1') and cast_bool(True)
    assert not cast_bool('off') and not cast_bool('0')
    with pytest.raises(ValueError):
        cast_bool('maybe')


def test_k8s_manifests_are_valid_settings():
    """deploy/k8s/*.yaml parse, and the autoscaler container's environment
    is a complete Settings (GPUMGR=k8s)."""
    import os
    import yaml
    from kiosk_autoscaler_amd.config import Config, Settings
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    docs = []
    for name in ('autoscaler.yaml', 'worker.yaml'):
        with open(os.path.join(root, 'deploy', 'k8s', name)) as handle:
            docs.extend(yaml.safe_load_all(handle))
    scaler = [d for d in docs if d['kind'] == 'Deployment' and
              d['metadata']['name'] == 'segmentation-autoscaler'][0]
    env = {e['name']: e['value'] for e in
           scaler['spec']['template']['spec']['containers'][0]['env']}
    s = Settings(Config(environ=env, use_files=False))
    assert s.GPUMGR == 'k8s' and s.MAX_PODS == 8
    worker = [d for d in docs if d['metadata']['name'] ==
              'segmentation-consumer'][0]
    assert worker['spec']['template']['spec']['containers'][0][
        'resources']['limits']['amd.com/gpu'] == 1
