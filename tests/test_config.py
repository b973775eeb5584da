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
