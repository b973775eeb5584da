"""Shared fixtures.  GPU tests carry ``@pytest.mark.gpu`` and run on MI355X."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (run via gpurun)')
    config.addinivalue_line('markers', 'slow: multi-second integration test')


@pytest.fixture
def engine():
    from kiosk_autoscaler_amd.fakes import RedisEngine
    return RedisEngine()


@pytest.fixture
def redis_client(engine):
    """The fakeredis.FakeStrictRedis analog of the reference's fixture."""
    from kiosk_autoscaler_amd.fakes import FakeRedis
    yield FakeRedis(engine=engine)


@pytest.fixture
def resp_server():
    from kiosk_autoscaler_amd.fakes import RespServer
    server = RespServer().start()
    yield server
    server.stop()


@pytest.fixture
def legacy_resp_server():
    """A RESP server answering as Redis 5.0 (the reference's
    ``redis~=3.5.3`` era): no LMOVE/BLMOVE, integer blocking timeouts."""
    from kiosk_autoscaler_amd.fakes import RedisEngine, RespServer
    server = RespServer(engine=RedisEngine(version='5.0.14')).start()
    yield server
    server.stop()


def kredis_binary():
    """``build/kredis-server``; ``KIOSK_KREDIS_BIN`` selects another build
    (CI runs the RESP suites against ``build/kredis-server-asan``)."""
    path = os.environ.get('KIOSK_KREDIS_BIN') or os.path.join(
        ROOT, 'build', 'kredis-server')
    return path if os.path.exists(path) else None


def _spawn_kredis(extra_args=()):
    """Start ``kredis-server`` on a free port; returns a handle or None."""
    import socket
    import subprocess
    import time
    binary = kredis_binary()
    if binary is None:
        return None
    sock = socket.socket()
    sock.bind(('127.0.0.1', 0))
    port = sock.getsockname()[1]
    sock.close()
    proc = subprocess.Popen([binary, '--port', str(port)] + list(extra_args),
                            stdout=subprocess.DEVNULL,
                            stderr=subprocess.DEVNULL)
    deadline = time.time() + 10
    while time.time() < deadline:
        try:
            socket.create_connection(('127.0.0.1', port), timeout=0.2).close()
            break
        except OSError:
            time.sleep(0.02)

    class Handle(object):
        host = '127.0.0.1'

    handle = Handle()
    handle.port = port
    handle.proc = proc
    return handle


def _stop_kredis(handle):
    import subprocess
    handle.proc.terminate()
    try:
        handle.proc.wait(timeout=5)
    except subprocess.TimeoutExpired:
        handle.proc.kill()


@pytest.fixture
def kredis_server():
    """The native C++ RESP server (skips if it has not been built)."""
    handle = _spawn_kredis()
    if handle is None:
        pytest.skip('kredis-server not built (python tools/build_native.py)')
    yield handle
    _stop_kredis(handle)


@pytest.fixture
def kredis_legacy_server():
    """``kredis-server --redis-version 5.0`` (skips if not built)."""
    handle = _spawn_kredis(['--redis-version', '5.0.14'])
    if handle is None:
        pytest.skip('kredis-server not built (python tools/build_native.py)')
    yield handle
    _stop_kredis(handle)
