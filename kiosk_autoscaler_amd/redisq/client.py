"""A compact synchronous Redis client (the subset the framework needs).

API shape follows the redis-py ``StrictRedis`` surface the reference uses
(``autoscaler/redis.py:158-161``: ``StrictRedis(host, port,
decode_responses=True, charset='utf-8')``; ``autoscaler/autoscaler.py:67-71``:
``llen``, ``scan_iter``) so the reference's call sites and the sentinel
retry proxy work unchanged on top of it.

Commands are methods that build an argument list and call
:meth:`Redis.execute_command`; per-command reply post-processing lives in
``RESPONSE_CALLBACKS``.  The transport is pluggable through the
``connection_pool`` argument: the in-process fake (``fakes.engine``) plugs a
loop-back pool in, so every reply callback is exercised identically against
the fake and against a real socket server.
"""
import threading

from . import exceptions
from .connection import ConnectionPool


def _bool_ok(reply):
    return reply == 'OK' or reply == b'OK' or reply is True


def _pairs_to_dict(reply):
    if not reply:
        return {}
    it = iter(reply)
    return dict(zip(it, it))


def _parse_info(reply):
    if isinstance(reply, bytes):
        reply = reply.decode('utf-8', 'replace')
    info = {}
    for line in (reply or '').splitlines():
        if not line or line.startswith('#') or ':' not in line:
            continue
        key, value = line.split(':', 1)
        info[key] = _coerce(value)
    return info


def _coerce(value):
    for cast in (int, float):
        try:
            return cast(value)
        except (TypeError, ValueError):
            pass
    return value


def _sentinel_state(flat):
    state = _pairs_to_dict(flat)
    for key in ('port', 'num-slaves', 'num-other-sentinels', 'quorum'):
        if key in state:
            state[key] = _coerce(state[key])
    flags = str(state.get('flags', ''))
    state['is_master'] = 'master' in flags
    state['is_slave'] = 'slave' in flags
    state['is_odown'] = 'o_down' in flags
    state['is_sdown'] = 's_down' in flags
    return state


def _parse_sentinel_masters(reply):
    result = {}
    for flat in reply or []:
        state = _sentinel_state(flat)
        result[state['name']] = state
    return result


def _parse_sentinel_slaves(reply):
    return [_sentinel_state(flat) for flat in reply or []]


def _parse_scan(reply):
    cursor, keys = reply
    return int(cursor), list(keys or [])


def _pop_pair(reply):
    return tuple(reply) if reply else None


RESPONSE_CALLBACKS = {
    'PING': lambda r: r in ('PONG', b'PONG') or r,
    'SET': lambda r: True if _bool_ok(r) else r,
    'MSET': _bool_ok,
    'HMSET': _bool_ok,
    'SELECT': _bool_ok,
    'FLUSHALL': _bool_ok,
    'FLUSHDB': _bool_ok,
    'RENAME': _bool_ok,
    'LSET': _bool_ok,
    'LTRIM': _bool_ok,
    'EXPIRE': bool,
    'PEXPIRE': bool,
    'PERSIST': bool,
    'HEXISTS': bool,
    'SISMEMBER': bool,
    'SETNX': bool,
    'HSETNX': bool,
    'HGETALL': _pairs_to_dict,
    'INFO': _parse_info,
    'SCAN': _parse_scan,
    'TIME': lambda r: (int(r[0]), int(r[1])),
    'BLPOP': _pop_pair,
    'BRPOP': _pop_pair,
    'SMEMBERS': lambda r: set(r or []),
    'SENTINEL MASTERS': _parse_sentinel_masters,
    'SENTINEL SLAVES': _parse_sentinel_slaves,
    'SENTINEL REPLICAS': _parse_sentinel_slaves,
    'SENTINEL GET-MASTER-ADDR-BY-NAME': lambda r: (r[0], int(r[1])) if r else None,
    'CLIENT SETNAME': _bool_ok,
    'SCRIPT FLUSH': _bool_ok,
    'SCRIPT KILL': _bool_ok,
}


class Redis(object):
    """Synchronous client. ``StrictRedis`` is an alias."""

    def __init__(self, host='localhost', port=6379, db=0, password=None,
                 socket_timeout=None, socket_connect_timeout=None,
                 decode_responses=False, encoding='utf-8', charset=None,
                 connection_pool=None, client_name=None, max_connections=64,
                 **_ignored):
        if charset is not None:  # legacy redis-py alias the reference passes
            encoding = charset
        if connection_pool is None:
            connection_pool = ConnectionPool(
                host=host, port=port, db=db, password=password,
                socket_timeout=socket_timeout,
                socket_connect_timeout=socket_connect_timeout,
                decode_responses=decode_responses, encoding=encoding,
                client_name=client_name, max_connections=max_connections)
        self.connection_pool = connection_pool
        self.response_callbacks = dict(RESPONSE_CALLBACKS)

    def __repr__(self):
        return '%s<%r>' % (type(self).__name__, self.connection_pool)

    # -- plumbing ----------------------------------------------------------
    def execute_command(self, *args, **options):
        """Send one command and return its post-processed reply."""
        pool = self.connection_pool
        conn = pool.get_connection()
        try:
            reply = self._roundtrip(conn, args, options)
        finally:
            pool.release(conn)
        return self._post(args, reply)

    @staticmethod
    def _roundtrip(conn, args, options):
        # like redis-py 3.5: a connection error disconnects and propagates;
        # retrying is the job of the RedisClient failover proxy above
        block_timeout = options.get('block_timeout')
        try:
            conn.send_command(*args)
            reply = conn.read_response(timeout=block_timeout)
        except exceptions.ConnectionError:
            conn.disconnect()
            raise
        if isinstance(reply, exceptions.RedisError):
            raise reply
        return reply

    def _post(self, args, reply):
        name = str(args[0]).upper()
        callback = None
        if len(args) > 1 and name in ('SENTINEL', 'CLIENT', 'SCRIPT',
                                      'CONFIG'):
            callback = self.response_callbacks.get(
                name + ' ' + str(args[1]).upper())
        if callback is None:
            callback = self.response_callbacks.get(name)
        return callback(reply) if callback else reply

    def pipeline(self, transaction=True):
        return Pipeline(self, transaction)

    def close(self):
        self.connection_pool.disconnect()

    # -- server --------------------------------------------------------------
    def ping(self):
        return self.execute_command('PING')

    def echo(self, value):
        return self.execute_command('ECHO', value)

    def time(self):
        return self.execute_command('TIME')

    def info(self, section=None):
        if section is None:
            return self.execute_command('INFO')
        return self.execute_command('INFO', section)

    def dbsize(self):
        return self.execute_command('DBSIZE')

    def flushdb(self):
        return self.execute_command('FLUSHDB')

    def flushall(self):
        return self.execute_command('FLUSHALL')

    def client_setname(self, name):
        return self.execute_command('CLIENT', 'SETNAME', name)

    def publish(self, channel, message):
        return self.execute_command('PUBLISH', channel, message)

    # -- keys ----------------------------------------------------------------
    def keys(self, pattern='*'):
        return self.execute_command('KEYS', pattern)

    def exists(self, *names):
        return self.execute_command('EXISTS', *names)

    def delete(self, *names):
        return self.execute_command('DEL', *names)

    def unlink(self, *names):
        return self.execute_command('UNLINK', *names)

    def type(self, name):
        return self.execute_command('TYPE', name)

    def expire(self, name, seconds):
        return self.execute_command('EXPIRE', name, int(seconds))

    def pexpire(self, name, millis):
        return self.execute_command('PEXPIRE', name, int(millis))

    def persist(self, name):
        return self.execute_command('PERSIST', name)

    def ttl(self, name):
        return self.execute_command('TTL', name)

    def pttl(self, name):
        return self.execute_command('PTTL', name)

    def rename(self, src, dst):
        return self.execute_command('RENAME', src, dst)

    def scan(self, cursor=0, match=None, count=None, _type=None):
        args = ['SCAN', cursor]
        if match is not None:
            args += ['MATCH', match]
        if count is not None:
            args += ['COUNT', count]
        if _type is not None:
            args += ['TYPE', _type]
        return self.execute_command(*args)

    def scan_iter(self, match=None, count=None, _type=None):
        """Generator over every key matching ``match`` (SCAN cursor walk).

        Like redis-py, the generator is lazy: errors raised while iterating
        happen outside any wrapper that merely returned it (the reference
        relies on that shape, ``autoscaler/autoscaler.py:70-71``)."""
        cursor = '0'
        while cursor != 0:
            cursor, keys = self.scan(cursor=cursor, match=match, count=count,
                                     _type=_type)
            for key in keys:
                yield key

    # -- strings -------------------------------------------------------------
    def get(self, name):
        return self.execute_command('GET', name)

    def set(self, name, value, ex=None, px=None, nx=False, xx=False):
        args = ['SET', name, value]
        if ex is not None:
            args += ['EX', int(ex)]
        if px is not None:
            args += ['PX', int(px)]
        if nx:
            args.append('NX')
        if xx:
            args.append('XX')
        return self.execute_command(*args)

    def setnx(self, name, value):
        return self.execute_command('SETNX', name, value)

    def mget(self, keys, *args):
        names = list(keys) if isinstance(keys, (list, tuple)) else [keys]
        return self.execute_command('MGET', *(names + list(args)))

    def mset(self, mapping):
        flat = []
        for key, value in mapping.items():
            flat += [key, value]
        return self.execute_command('MSET', *flat)

    def incr(self, name, amount=1):
        return self.execute_command('INCRBY', name, amount)

    incrby = incr

    def decr(self, name, amount=1):
        return self.execute_command('DECRBY', name, amount)

    # -- lists ---------------------------------------------------------------
    def lpush(self, name, *values):
        return self.execute_command('LPUSH', name, *values)

    def rpush(self, name, *values):
        return self.execute_command('RPUSH', name, *values)

    def lpop(self, name, count=None):
        if count is None:
            return self.execute_command('LPOP', name)
        return self.execute_command('LPOP', name, count)

    def rpop(self, name, count=None):
        if count is None:
            return self.execute_command('RPOP', name)
        return self.execute_command('RPOP', name, count)

    def llen(self, name):
        return self.execute_command('LLEN', name)

    def lrange(self, name, start, end):
        return self.execute_command('LRANGE', name, start, end)

    def lindex(self, name, index):
        return self.execute_command('LINDEX', name, index)

    def lrem(self, name, count, value):
        return self.execute_command('LREM', name, count, value)

    def ltrim(self, name, start, end):
        return self.execute_command('LTRIM', name, start, end)

    def lset(self, name, index, value):
        return self.execute_command('LSET', name, index, value)

    def lmove(self, first_list, second_list, src='LEFT', dest='RIGHT'):
        return self.execute_command('LMOVE', first_list, second_list, src,
                                    dest)

    def blmove(self, first_list, second_list, timeout, src='LEFT',
               dest='RIGHT'):
        return self.execute_command(
            'BLMOVE', first_list, second_list, src, dest, timeout,
            block_timeout=_block_deadline(timeout))

    def rpoplpush(self, src, dst):
        return self.execute_command('RPOPLPUSH', src, dst)

    def brpoplpush(self, src, dst, timeout=0):
        return self.execute_command('BRPOPLPUSH', src, dst, timeout,
                                    block_timeout=_block_deadline(timeout))

    def blpop(self, keys, timeout=0):
        keys = [keys] if isinstance(keys, (str, bytes)) else list(keys)
        return self.execute_command('BLPOP', *(keys + [timeout]),
                                    block_timeout=_block_deadline(timeout))

    def brpop(self, keys, timeout=0):
        keys = [keys] if isinstance(keys, (str, bytes)) else list(keys)
        return self.execute_command('BRPOP', *(keys + [timeout]),
                                    block_timeout=_block_deadline(timeout))

    # -- hashes --------------------------------------------------------------
    def hset(self, name, key=None, value=None, mapping=None):
        flat = []
        if key is not None:
            flat += [key, value]
        for k, v in (mapping or {}).items():
            flat += [k, v]
        if not flat:
            raise exceptions.DataError("'hset' with no key value pairs")
        return self.execute_command('HSET', name, *flat)

    def hmset(self, name, mapping):
        flat = []
        for k, v in mapping.items():
            flat += [k, v]
        return self.execute_command('HMSET', name, *flat)

    def hsetnx(self, name, key, value):
        return self.execute_command('HSETNX', name, key, value)

    def hget(self, name, key):
        return self.execute_command('HGET', name, key)

    def hmget(self, name, keys, *args):
        names = list(keys) if isinstance(keys, (list, tuple)) else [keys]
        return self.execute_command('HMGET', name, *(names + list(args)))

    def hgetall(self, name):
        return self.execute_command('HGETALL', name)

    def hdel(self, name, *keys):
        return self.execute_command('HDEL', name, *keys)

    def hlen(self, name):
        return self.execute_command('HLEN', name)

    def hexists(self, name, key):
        return self.execute_command('HEXISTS', name, key)

    def hincrby(self, name, key, amount=1):
        return self.execute_command('HINCRBY', name, key, amount)

    def hkeys(self, name):
        return self.execute_command('HKEYS', name)

    def hvals(self, name):
        return self.execute_command('HVALS', name)

    # -- sets ----------------------------------------------------------------
    def sadd(self, name, *values):
        return self.execute_command('SADD', name, *values)

    def srem(self, name, *values):
        return self.execute_command('SREM', name, *values)

    def smembers(self, name):
        return self.execute_command('SMEMBERS', name)

    def scard(self, name):
        return self.execute_command('SCARD', name)

    def sismember(self, name, value):
        return self.execute_command('SISMEMBER', name, value)

    # -- scripting -------------------------------------------------------------
    def eval(self, script, numkeys, *keys_and_args):
        return self.execute_command('EVAL', script, numkeys, *keys_and_args)

    def evalsha(self, sha, numkeys, *keys_and_args):
        return self.execute_command('EVALSHA', sha, numkeys, *keys_and_args)

    def script_load(self, script):
        return self.execute_command('SCRIPT', 'LOAD', script)

    def script_kill(self):
        return self.execute_command('SCRIPT', 'KILL')

    # -- sentinel ------------------------------------------------------------
    def sentinel_masters(self):
        return self.execute_command('SENTINEL', 'MASTERS')

    def sentinel_slaves(self, service_name):
        return self.execute_command('SENTINEL', 'SLAVES', service_name)

    def sentinel_get_master_addr_by_name(self, service_name):
        return self.execute_command('SENTINEL', 'GET-MASTER-ADDR-BY-NAME',
                                    service_name)


StrictRedis = Redis


def _block_deadline(timeout):
    """Socket read timeout for a blocking command (0 = block forever)."""
    try:
        timeout = float(timeout)
    except (TypeError, ValueError):
        return None
    if timeout <= 0:
        return None
    return timeout + 5.0


class Pipeline(object):
    """Buffers commands and sends them in one round trip.

    With ``transaction=True`` the batch is wrapped in MULTI/EXEC so the server
    applies it atomically (used by the race-free tally)."""

    def __init__(self, client, transaction=True):
        self.client = client
        self.transaction = transaction
        self._stack = []
        self._lock = threading.Lock()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.reset()

    def reset(self):
        self._stack = []

    def __len__(self):
        return len(self._stack)

    def execute_command(self, *args, **_options):
        self._stack.append(args)
        return self

    def __getattr__(self, name):
        # reuse the client's command builders, redirected into the buffer
        method = getattr(Redis, name, None)
        if method is None or name.startswith('_') or name in (
                'pipeline', 'scan_iter', 'close'):
            raise AttributeError(name)

        def queued(*args, **kwargs):
            return method(self, *args, **kwargs)
        return queued

    def execute(self, raise_on_error=True):
        commands = list(self._stack)
        self._stack = []
        if not commands:
            return []
        if self.transaction:
            wire = [('MULTI',)] + commands + [('EXEC',)]
        else:
            wire = commands
        pool = self.client.connection_pool
        conn = pool.get_connection()
        try:
            conn.send_commands(wire)
            replies = [conn.read_response() for _ in wire]
        except exceptions.ConnectionError:
            conn.disconnect()
            raise
        finally:
            pool.release(conn)
        if self.transaction:
            queued_errors = [r for r in replies[1:-1]
                             if isinstance(r, exceptions.RedisError)]
            result = replies[-1]
            if isinstance(result, exceptions.RedisError):
                raise (queued_errors[0] if queued_errors else result)
            if result is None:
                raise exceptions.ResponseError('transaction aborted (WATCH)')
        else:
            result = replies
        out = []
        for args, reply in zip(commands, result):
            if isinstance(reply, exceptions.RedisError):
                if raise_on_error:
                    raise reply
                out.append(reply)
            else:
                out.append(self.client._post(args, reply))
        return out
