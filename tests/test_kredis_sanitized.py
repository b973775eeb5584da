"""kredis-server under AddressSanitizer + UndefinedBehaviorSanitizer
(the 1 200-line epoll/RESP C++ server had no
sanitizer run).  The ASan build (``tools/build_native.py --sanitize``) is
driven with the client's real command mix, the blocking moves, the SCAN
paging, MULTI/EXEC -- and with malformed and hostile RESP frames (truncated
bulks, negative/huge lengths, garbage types, deep arrays, binary noise).
The server must keep serving, and on SIGTERM exit cleanly with no ASan,
UBSan or LeakSanitizer report.  CPU only (host code; no GPU sanitizer)."""
import glob
import os
import random
import shutil
import socket
import subprocess
import sys
import threading
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow


@pytest.fixture(scope='module')
def asan_server(tmp_path_factory):
    if shutil.which('g++') is None:
        pytest.skip('no g++')
    sys.path.insert(0, os.path.join(ROOT, 'tools'))
    import build_native
    binary = build_native.build_kredis(sanitize=True)
    logs = tmp_path_factory.mktemp('asan')
    sock = socket.socket()
    sock.bind(('127.0.0.1', 0))
    port = sock.getsockname()[1]
    sock.close()
    env = dict(os.environ,
               ASAN_OPTIONS='detect_leaks=1:abort_on_error=0:log_path=%s/asan'
               % logs,
               UBSAN_OPTIONS='print_stacktrace=1:halt_on_error=1:'
               'log_path=%s/ubsan' % logs)
    proc = subprocess.Popen([binary, '--port', str(port)], env=env,
                            stdout=subprocess.DEVNULL,
                            stderr=subprocess.PIPE)
    deadline = time.time() + 20
    while time.time() < deadline:
        try:
            socket.create_connection(('127.0.0.1', port), timeout=0.2).close()
            break
        except OSError:
            time.sleep(0.05)

    class Handle(object):
        host = '127.0.0.1'
    handle = Handle()
    handle.port = port
    handle.proc = proc
    handle.logs = logs
    yield handle
    if proc.poll() is None:
        proc.kill()


def _client(server):
    from kiosk_autoscaler_amd.redisq import StrictRedis
    return StrictRedis(host=server.host, port=server.port,
                       decode_responses=True)


def test_command_mix(asan_server):
    c = _client(asan_server)
    assert c.ping()
    c.set('s', 'v', ex=100)
    assert c.get('s') == 'v' and 0 < c.ttl('s') <= 100
    c.hset('h', mapping={'a': '1', 'b': '2'})
    assert c.hgetall('h') == {'a': '1', 'b': '2'}
    for i in range(50):
        c.lpush('q', 'item%d' % i)
    for i in range(10):
        assert c.lmove('q', 'processing-q:w-g0-a-%d' % i, 'RIGHT', 'LEFT')
    assert c.llen('q') == 40
    assert len(list(c.scan_iter(match='processing-q:*', count=3))) == 10
    pipe = c.pipeline(transaction=True)
    pipe.llen('q')
    pipe.keys('processing-q:*')
    waiting, keys = pipe.execute()
    assert waiting == 40 and len(keys) == 10
    assert c.delete(*keys) == 10
    assert c.expire('h', 1)
    c.rpoplpush('q', 'q2')
    assert c.lrange('q2', 0, -1)

    # a blocked BLMOVE woken by a producer on another connection
    got = {}

    def consumer():
        got['v'] = _client(asan_server).blmove('empty', 'dst', 5, 'RIGHT',
                                               'LEFT')
    th = threading.Thread(target=consumer)
    th.start()
    time.sleep(0.1)
    c.lpush('empty', 'x')
    th.join(10)
    assert got['v'] == 'x'


def _raw(server, payload, read=True):
    sock = socket.create_connection((server.host, server.port), timeout=2)
    try:
        sock.sendall(payload)
        if read:
            try:
                return sock.recv(4096)
            except socket.timeout:
                return b''
        return b''
    finally:
        sock.close()


HOSTILE = [
    b'*1\r\n$4\r\nPING\r\n',                      # valid
    b'*2\r\n$3\r\nGET\r\n$-5\r\n',               # negative bulk length
    b'*1\r\n$99999999999\r\nPING\r\n',            # absurd bulk length
    b'*-3\r\n',                                   # negative array
    b'*3\r\n$3\r\nSET\r\n$1\r\nk\r\n',            # truncated array
    b'*2\r\n$3\r\nGET\r\n$10\r\nshort\r\n',       # bulk shorter than said
    b'*1\r\n:12\r\n',                             # integer as argument
    b'?weird\r\n',                                # unknown type byte
    b'PING\r\nECHO hello\r\n',                    # inline commands
    b'*1\r\n$0\r\n\r\n',                          # empty command name
    b'*4\r\n$4\r\nSCAN\r\n$2\r\n-1\r\n$5\r\nCOUNT\r\n$1\r\n0\r\n',
    b'*3\r\n$6\r\nLRANGE\r\n$1\r\nq\r\n$3\r\nabc\r\n',   # missing arg
    b'*2\r\n$6\r\nEXPIRE\r\n$1\r\nq\r\n',         # too few arguments
    b'*1\r\n$4\r\nEXEC\r\n',                      # EXEC without MULTI
    b'*1\r\n$7\r\nUNKNOWN\r\n',
    b'*1000000\r\n',                              # huge array header
    b'\x00\xff\r\n' * 64,
]


def test_hostile_frames_do_not_break_the_server(asan_server):
    rng = random.Random(7)
    frames = list(HOSTILE)
    for _ in range(200):                          # random noise and splices
        n = rng.randrange(1, 200)
        noise = bytes(rng.randrange(256) for _ in range(n))
        base = rng.choice(HOSTILE)
        cut = rng.randrange(len(base) + 1)
        frames.append(base[:cut] + noise)
    for frame in frames:
        _raw(asan_server, frame, read=False)
    # deeply nested arrays are rejected, not recursed into
    _raw(asan_server, b'*1\r\n' * 10000, read=False)
    # byte-at-a-time delivery of a valid command still parses
    sock = socket.create_connection((asan_server.host, asan_server.port))
    for byte in b'*1\r\n$4\r\nPING\r\n':
        sock.send(bytes([byte]))
        time.sleep(0.001)
    assert sock.recv(64).startswith(b'+PONG')
    sock.close()
    assert asan_server.proc.poll() is None
    assert _client(asan_server).ping()


def test_clean_exit_without_sanitizer_reports(asan_server):
    proc = asan_server.proc
    assert proc.poll() is None
    proc.terminate()                     # graceful: LeakSanitizer runs
    _, err = proc.communicate(timeout=60)
    reports = []
    for path in glob.glob(str(asan_server.logs / '*')):
        with open(path) as handle:
            reports.append(handle.read())
    text = '\n'.join(reports) + err.decode(errors='replace')
    assert 'ERROR: AddressSanitizer' not in text, text[-4000:]
    assert 'ERROR: LeakSanitizer' not in text, text[-4000:]
    assert 'runtime error' not in text, text[-4000:]
    assert proc.returncode == 0, text[-4000:]
