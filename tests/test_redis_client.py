"""RESP codec, client reply callbacks, in-proc engine and socket servers."""
import threading
import time

import pytest

from kiosk_autoscaler_amd.fakes import FakeRedis, RedisEngine, glob_match
from kiosk_autoscaler_amd.redisq import StrictRedis, exceptions
from kiosk_autoscaler_amd.redisq.resp import (NOT_READY, ReplyError,
                                              RespParser, encode_command,
                                              encode_reply)


def test_encode_command():
    assert encode_command('LLEN', 'q') == b'*2\r\n$4\r\nLLEN\r\n$1\r\nq\r\n'
    assert encode_command('SET', 'k', 12) == \
        b'*3\r\n$3\r\nSET\r\n$1\r\nk\r\n$2\r\n12\r\n'
    with pytest.raises(exceptions.DataError):
        encode_command('SET', 'k', True)


def test_parser_incremental_and_nested():
    data = encode_reply([1, b'ab', None, [b'x', ReplyError('ERR no')]])
    parser = RespParser(decode=True)
    for i in range(len(data) - 1):   # byte by byte: never a partial reply
        parser.feed(data[i:i + 1])
        assert parser.gets() is NOT_READY
    parser.feed(data[-1:])
    reply = parser.gets()
    assert reply[:3] == [1, 'ab', None]
    assert reply[3][0] == 'x' and isinstance(reply[3][1], ReplyError)
    assert parser.gets() is NOT_READY


def test_glob():
    assert glob_match(b'processing-predict:*', b'processing-predict:h1')
    assert not glob_match(b'processing-predict:*', b'processing-predict')
    assert glob_match(b'a?c', b'abc') and glob_match(b'[ab]x', b'bx')


def _exercise(client):
    assert client.ping() is True
    assert client.lpush('q', 'a', 'b', 'c') == 3
    assert client.llen('q') == 3
    assert client.lrange('q', 0, -1) == ['c', 'b', 'a']
    assert client.lmove('q', 'processing-q:w1', 'RIGHT', 'LEFT') == 'a'
    assert client.rpoplpush('q', 'processing-q:w2') == 'b'
    assert sorted(client.scan_iter(match='processing-q:*', count=1)) == [
        'processing-q:w1', 'processing-q:w2']
    assert client.delete('processing-q:w1', 'nope') == 1
    assert client.hset('job', mapping={'rows': 4, 'status': 'new'}) == 2
    assert client.hgetall('job') == {'rows': '4', 'status': 'new'}
    assert client.hmset('job', {'status': 'done'}) is True
    assert client.hget('job', 'status') == 'done'
    assert client.set('k', 'v', ex=10) is True
    assert 0 < client.ttl('k') <= 10
    assert client.get('k') == 'v'
    assert client.type('job') == 'hash'
    assert client.exists('k', 'job', 'zz') == 2
    assert client.incr('n') == 1 and client.incr('n', 5) == 6
    info = client.info()
    assert 'redis_version' in info
    with pytest.raises(exceptions.ResponseError):
        client.lpush('k', 'x')          # WRONGTYPE
    with pytest.raises(exceptions.ResponseError):
        client.sentinel_masters()       # plain redis: unknown command
    pipe = client.pipeline()
    pipe.llen('q').lpush('q', 'z').llen('q')
    assert pipe.execute() == [1, 2, 2]
    assert client.blmove('empty', 'dst', 0.05) is None
    assert client.blpop(['empty'], timeout=0.05) is None


def test_fake_client(redis_client):
    _exercise(redis_client)


def test_python_server(resp_server):
    client = StrictRedis(host=resp_server.host, port=resp_server.port,
                         decode_responses=True)
    _exercise(client)


def test_native_server(kredis_server):
    client = StrictRedis(host=kredis_server.host, port=kredis_server.port,
                         decode_responses=True)
    client.flushall()
    _exercise(client)


def test_blocking_move_wakes(resp_server):
    host, port = resp_server.host, resp_server.port
    consumer = StrictRedis(host=host, port=port, decode_responses=True)
    producer = StrictRedis(host=host, port=port, decode_responses=True)
    got = {}

    def consume():
        t0 = time.monotonic()
        got['item'] = consumer.blmove('jobs', 'processing-jobs:w', 5,
                                      'RIGHT', 'LEFT')
        got['dt'] = time.monotonic() - t0
    thread = threading.Thread(target=consume)
    thread.start()
    time.sleep(0.1)
    producer.lpush('jobs', 'j1')
    thread.join(5)
    assert got['item'] == 'j1'
    assert got['dt'] < 1.0
    assert producer.lrange('processing-jobs:w', 0, -1) == ['j1']


def test_connection_refused():
    client = StrictRedis(host='127.0.0.1', port=1, socket_connect_timeout=0.5)
    with pytest.raises(exceptions.ConnectionError):
        client.ping()


def test_fault_injection_engine():
    engine = RedisEngine()
    client = FakeRedis(engine=engine)
    engine.inject_fault('LLEN', 'connection')
    with pytest.raises(exceptions.ConnectionError):
        client.llen('q')
    assert client.llen('q') == 0                 # one-shot
    engine.inject_fault('LLEN', 'busy')
    with pytest.raises(exceptions.ResponseError) as info:
        client.llen('q')
    assert 'BUSY' in str(info.value) and 'SCRIPT KILL' in str(info.value)


def test_expiry_and_scan_type(redis_client):
    redis_client.set('short', '1', px=30)
    redis_client.rpush('l', 'x')
    time.sleep(0.06)
    assert redis_client.get('short') is None
    assert list(redis_client.scan_iter(_type='list')) == ['l']


def test_native_sentinel_personality():
    """kredis in sentinel mode + data node: RedisClient discovery end to end."""
    import socket
    import subprocess
    from unittest import mock
    from conftest import kredis_binary
    from kiosk_autoscaler_amd.redisq import RedisClient
    binary = kredis_binary()
    if binary is None:
        pytest.skip('kredis-server not built')

    def port():
        s = socket.socket()
        s.bind(('127.0.0.1', 0))
        p = s.getsockname()[1]
        s.close()
        return p
    data_port, sentinel_port = port(), port()
    procs = [subprocess.Popen([binary, '--port', str(data_port)],
                              stdout=subprocess.DEVNULL),
             subprocess.Popen([binary, '--port', str(sentinel_port),
                               '--sentinel', 'mymaster', '127.0.0.1',
                               str(data_port), '--replica',
                               '127.0.0.1:%d' % data_port],
                              stdout=subprocess.DEVNULL)]
    try:
        for p in (data_port, sentinel_port):
            deadline = time.time() + 10
            while time.time() < deadline:
                try:
                    socket.create_connection(('127.0.0.1', p), 0.2).close()
                    break
                except OSError:
                    time.sleep(0.02)
        client = RedisClient('127.0.0.1', sentinel_port, backoff=0)
        assert client._redis_master is not client._sentinel
        assert len(client._redis_slaves) == 1
        client.lpush('predict', 'a', 'b')
        assert client.llen('predict') == 2          # via the replica
        assert client._sentinel.sentinel_get_master_addr_by_name(
            'mymaster') == ('127.0.0.1', data_port)
        with mock.patch('time.sleep'):
            pass
    finally:
        for p in procs:
            p.terminate()
            p.wait(timeout=5)


def test_native_scan_survives_deletes_between_pages(kredis_server):
    """SCAN guarantee: a key present for the whole scan is
    returned even when keys already returned are deleted between pages
    (kredis's cursor is a hash position, not an index)."""
    client = StrictRedis(host=kredis_server.host, port=kredis_server.port,
                         decode_responses=True)
    names = ['processing-q:w-%04d' % i for i in range(3000)]
    pipe = client.pipeline(transaction=False)
    for name in names:
        pipe.rpush(name, 'x')
    pipe.execute()
    seen, deleted = set(), set()
    cursor = 0
    while True:
        cursor, page = client.scan(cursor, match='processing-q:*', count=97)
        seen.update(page)
        # workers complete items: delete some of what was already returned
        victims = sorted(seen - deleted)[:13]
        if victims:
            client.delete(*victims)
            deleted.update(victims)
        if int(cursor) == 0:
            break
    assert set(names) - deleted <= seen
    assert len(seen) == len(names)          # never duplicated either


def test_native_server_redis5_mode(kredis_legacy_server):
    """``kredis-server --redis-version 5.0``: LMOVE/BLMOVE are unknown,
    blocking timeouts must be integers, SCAN ignores TYPE -- and the
    worker's consumer still pulls in FIFO order through RPOPLPUSH."""
    from kiosk_autoscaler_amd.worker.runtime import QueueConsumer
    client = StrictRedis(host=kredis_legacy_server.host,
                         port=kredis_legacy_server.port,
                         decode_responses=True)
    assert client.info()['redis_version'].startswith('5.0')
    with pytest.raises(exceptions.ResponseError, match='unknown command'):
        client.lmove('q', 'p', 'RIGHT', 'LEFT')
    with pytest.raises(exceptions.ResponseError, match='not an integer'):
        client.brpoplpush('q', 'p', 0.005)
    assert client.brpoplpush('q', 'p', 1) is None       # integer: fine
    consumer = QueueConsumer(client, 'w-g0-x-9', ['q'], poll_block=0.005)
    assert consumer.pull(limit=1) == []
    assert (consumer.move_mode, consumer.block_mode) == ('rpoplpush', 'poll')
    client.lpush('q', 'a', 'b')
    taken = [consumer.pull(limit=1)[0][1] for _ in range(2)]
    assert taken == ['a', 'b']
