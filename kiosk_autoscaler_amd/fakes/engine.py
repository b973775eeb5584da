"""In-process Redis data engine (replaces ``fakeredis`` for tests).

The reference's tests run against ``fakeredis.FakeStrictRedis``
(``autoscaler/autoscaler_test.py:40-42``) and fake a sentinel cluster by
sub-classing it (``autoscaler/redis_test.py:41-68``).  Neither fakeredis nor
a redis-server binary exists in this environment, so the
framework ships its own engine:

* :class:`RedisEngine` executes RESP command arrays against typed keyspaces
  (strings, lists, hashes, sets), with TTLs, glob ``KEYS``/``SCAN``,
  ``MULTI``/``EXEC``, blocking list moves, a ``SENTINEL`` personality and a
  fault-injection hook (drop the connection / answer ``BUSY``).
* :class:`FakeRedis` is the real :class:`~kiosk_autoscaler_amd.redisq.Redis`
  client wired to an engine through a loop-back connection that round-trips
  every reply through the RESP encoder and parser, so client reply
  callbacks run exactly as they do over a socket.
"""
import fnmatch
import re
import threading
import time

from ..redisq import exceptions
from ..redisq.client import Redis
from ..redisq.resp import (NOT_READY, NULL_ARRAY, ReplyError, RespParser,
                           SimpleString, encode_reply)

OK = SimpleString('OK')
WRONGTYPE = ReplyError(
    'WRONGTYPE Operation against a key holding the wrong kind of value')
BUSY_MESSAGE = ('BUSY Redis is busy running a script. You can only call '
                'SCRIPT KILL or SHUTDOWN NOSCRIPT.')


class DropConnection(Exception):
    """Raised inside the engine to make the transport drop the client."""


def _b(value):
    if isinstance(value, bytes):
        return value
    if isinstance(value, str):
        return value.encode('utf-8')
    return str(value).encode('utf-8')


def _int(value):
    try:
        return int(value)
    except (TypeError, ValueError):
        raise _Reply(ReplyError('ERR value is not an integer or out of range'))


def _float(value):
    try:
        return float(value)
    except (TypeError, ValueError):
        raise _Reply(ReplyError('ERR timeout is not a float or out of range'))


def parse_version(text):
    """``'5.0.14'`` -> ``(5, 0, 14)``."""
    parts = []
    for piece in str(text).split('-')[0].split('.'):
        try:
            parts.append(int(piece))
        except ValueError:
            break
    return tuple(parts) or (7, 2, 0)


class _Reply(Exception):
    """Short-circuit a handler with a ready reply (usually an error)."""

    def __init__(self, reply):
        Exception.__init__(self)
        self.reply = reply


_GLOB_CACHE = {}


def glob_match(pattern, key):
    """Redis-style glob (``* ? [..] \\x``) over bytes."""
    regex = _GLOB_CACHE.get(pattern)
    if regex is None:
        text = fnmatch.translate(pattern.decode('latin-1'))
        regex = re.compile(text.encode('latin-1'), re.DOTALL)
        if len(_GLOB_CACHE) < 1024:
            _GLOB_CACHE[pattern] = regex
    return regex.match(key) is not None


class Session(object):
    """Per-connection state: selected db, MULTI queue, client name."""

    __slots__ = ('db', 'multi', 'name', 'closed')

    def __init__(self):
        self.db = 0
        self.multi = None
        self.name = None
        self.closed = False


class RedisEngine(object):
    """Thread-safe keyspace engine.

    Args:
        sentinel_masters: optional ``{name: {'ip':..., 'port':...,
            'replicas': [(ip, port), ...]}}``; when given the engine answers
            ``SENTINEL MASTERS/SLAVES/GET-MASTER-ADDR-BY-NAME`` like a
            sentinel.  Without it ``SENTINEL`` is an unknown command, which
            is what a plain Redis answers (reference ``redis.py:153-155``
            path).
        databases: number of logical dbs.
        version: the Redis version to answer as (``INFO``'s
            ``redis_version``).  Below 6.2 ``LMOVE``/``BLMOVE`` are unknown
            commands; below 6.0 a blocking timeout must be an integer and
            ``SCAN`` has no ``TYPE`` option -- what a server of the
            reference's ``redis~=3.5.3`` era (``requirements.txt:3``) does.
    """

    # first version with the command (absent from this engine's older modes)
    SINCE = {'LMOVE': (6, 2), 'BLMOVE': (6, 2)}

    def __init__(self, sentinel_masters=None, databases=16,
                 version='7.2.0'):
        self.version_text = str(version)
        self.version = parse_version(version)
        self._dbs = [dict() for _ in range(databases)]
        self._expires = [dict() for _ in range(databases)]
        self._cond = threading.Condition(threading.RLock())
        self.sentinel_masters = sentinel_masters
        self._faults = []  # [command, kind, remaining]
        self.commands_processed = 0
        self.started = time.time()
        self._handlers = self._build_table()

    # -- fault injection ----------------------------------------------------
    def inject_fault(self, command, kind='connection', times=1):
        """Make the next ``times`` calls of ``command`` fail.

        ``kind``: ``'connection'`` (drop the client), ``'busy'`` (BUSY
        script error) or ``'error'`` (generic ERR)."""
        with self._cond:
            self._faults.append([command.upper(), kind, int(times)])

    def clear_faults(self):
        with self._cond:
            self._faults = []

    def _take_fault(self, name):
        for fault in self._faults:
            if fault[0] in (name, '*') and fault[2] > 0:
                fault[2] -= 1
                return fault[1]
        return None

    # -- keyspace helpers ------------------------------------------------------
    def _db(self, session):
        return self._dbs[session.db]

    def _alive(self, session, key):
        expires = self._expires[session.db]
        deadline = expires.get(key)
        if deadline is not None and time.monotonic() >= deadline:
            del expires[key]
            self._dbs[session.db].pop(key, None)
            return False
        return key in self._dbs[session.db]

    def _get(self, session, key, kind):
        if not self._alive(session, key):
            return None
        value = self._dbs[session.db][key]
        if not isinstance(value, kind):
            raise _Reply(WRONGTYPE)
        return value

    def _get_or_create(self, session, key, kind):
        value = self._get(session, key, kind)
        if value is None:
            value = kind()
            self._dbs[session.db][key] = value
        return value

    def _drop_if_empty(self, session, key, value):
        if not value:
            self._dbs[session.db].pop(key, None)
            self._expires[session.db].pop(key, None)

    def _delete(self, session, key):
        self._expires[session.db].pop(key, None)
        return self._dbs[session.db].pop(key, None) is not None

    def _live_keys(self, session):
        return [k for k in list(self._dbs[session.db]) if self._alive(session, k)]

    # -- dispatch ------------------------------------------------------------
    def execute(self, session, args):
        """Run one command (list of bytes/str) and return a reply value."""
        if not args:
            return ReplyError('ERR empty command')
        args = [_b(a) for a in args]
        name = args[0].decode('latin-1').upper()
        with self._cond:
            fault = self._take_fault(name)
        if fault == 'connection':
            raise DropConnection(name)
        if fault == 'busy':
            return ReplyError(BUSY_MESSAGE)
        if fault == 'error':
            return ReplyError('ERR injected failure')
        if session.multi is not None and name not in ('EXEC', 'DISCARD',
                                                      'MULTI', 'WATCH'):
            if name not in self._handlers:
                return ReplyError("ERR unknown command '%s'" % name.lower())
            session.multi.append(args)
            return SimpleString('QUEUED')
        handler = self._handlers.get(name)
        if handler is None:
            return ReplyError("ERR unknown command '%s', with args beginning "
                              "with: " % args[0].decode('latin-1'))
        try:
            if name in self._BLOCKING:
                return handler(session, args[1:])
            with self._cond:
                self.commands_processed += 1
                reply = handler(session, args[1:])
                if name in self._WAKES:
                    self._cond.notify_all()
                return reply
        except _Reply as short:
            return short.reply
        except (IndexError, ValueError):
            return ReplyError("ERR wrong number of arguments for '%s' command"
                              % name.lower())

    _BLOCKING = frozenset(['BLMOVE', 'BRPOPLPUSH', 'BLPOP', 'BRPOP'])
    _WAKES = frozenset(['LPUSH', 'RPUSH', 'LMOVE', 'RPOPLPUSH', 'EXEC',
                        'RENAME', 'LPUSHX', 'RPUSHX'])

    def _build_table(self):
        table = {}
        for attr in dir(self):
            if attr.startswith('cmd_'):
                name = attr[4:].upper().replace('_', '-')
                if self.version >= self.SINCE.get(name, (0,)):
                    table[name] = getattr(self, attr)
        return table

    def _timeout(self, value):
        """A blocking command's timeout: fractional only since 6.0."""
        if self.version < (6, 0):
            try:
                return float(int(value))
            except (TypeError, ValueError):
                raise _Reply(ReplyError(
                    'ERR timeout is not an integer or out of range'))
        return _float(value)

    # -- connection / server -------------------------------------------------
    def cmd_ping(self, session, args):
        return args[0] if args else SimpleString('PONG')

    def cmd_echo(self, session, args):
        return args[0]

    def cmd_select(self, session, args):
        index = _int(args[0])
        if not 0 <= index < len(self._dbs):
            return ReplyError('ERR DB index is out of range')
        session.db = index
        return OK

    def cmd_auth(self, session, args):
        return OK

    def cmd_quit(self, session, args):
        session.closed = True
        return OK

    def cmd_dbsize(self, session, args):
        return len(self._live_keys(session))

    def cmd_flushdb(self, session, args):
        self._dbs[session.db].clear()
        self._expires[session.db].clear()
        return OK

    def cmd_flushall(self, session, args):
        for db, exp in zip(self._dbs, self._expires):
            db.clear()
            exp.clear()
        return OK

    def cmd_time(self, session, args):
        now = time.time()
        return [str(int(now)).encode(), str(int((now % 1) * 1e6)).encode()]

    def cmd_info(self, session, args):
        keyspace = ''.join(
            'db%d:keys=%d,expires=%d\r\n' % (i, len(db), len(self._expires[i]))
            for i, db in enumerate(self._dbs) if db)
        role = 'sentinel' if self.sentinel_masters else 'master'
        text = ('# Server\r\nredis_version:%s-kiosk-amd\r\n'
                'redis_mode:%s\r\nuptime_in_seconds:%d\r\n'
                '# Replication\r\nrole:%s\r\n'
                '# Stats\r\ntotal_commands_processed:%d\r\n'
                '# Keyspace\r\n%s' % (
                    self.version_text,
                    'sentinel' if self.sentinel_masters else 'standalone',
                    int(time.time() - self.started), role,
                    self.commands_processed, keyspace))
        return text.encode()

    def cmd_client(self, session, args):
        sub = args[0].upper()
        if sub == b'SETNAME':
            session.name = args[1]
            return OK
        if sub == b'GETNAME':
            return session.name
        if sub == b'ID':
            return id(session) & 0x7FFFFFFF
        return OK

    def cmd_command(self, session, args):
        return []

    def cmd_config(self, session, args):
        return []

    # -- transactions --------------------------------------------------------
    def cmd_multi(self, session, args):
        if session.multi is not None:
            return ReplyError('ERR MULTI calls can not be nested')
        session.multi = []
        return OK

    def cmd_discard(self, session, args):
        if session.multi is None:
            return ReplyError('ERR DISCARD without MULTI')
        session.multi = None
        return OK

    def cmd_exec(self, session, args):
        if session.multi is None:
            return ReplyError('ERR EXEC without MULTI')
        queued, session.multi = session.multi, None
        results = []
        for cmd in queued:
            name = cmd[0].decode('latin-1').upper()
            try:
                results.append(self._handlers[name](session, cmd[1:]))
            except _Reply as short:
                results.append(short.reply)
            except (IndexError, ValueError):
                results.append(ReplyError('ERR wrong number of arguments'))
        return results

    def cmd_watch(self, session, args):
        return OK

    def cmd_unwatch(self, session, args):
        return OK

    # -- generic keys ----------------------------------------------------------
    def cmd_keys(self, session, args):
        pattern = args[0]
        return sorted(k for k in self._live_keys(session)
                      if glob_match(pattern, k))

    def cmd_exists(self, session, args):
        return sum(1 for k in args if self._alive(session, k))

    def cmd_del(self, session, args):
        return sum(1 for k in args if self._alive(session, k)
                   and self._delete(session, k))

    cmd_unlink = cmd_del

    def cmd_type(self, session, args):
        if not self._alive(session, args[0]):
            return SimpleString('none')
        value = self._db(session)[args[0]]
        return SimpleString({bytes: 'string', list: 'list', dict: 'hash',
                             set: 'set'}[type(value)])

    def _set_deadline(self, session, key, seconds):
        if not self._alive(session, key):
            return 0
        self._expires[session.db][key] = time.monotonic() + seconds
        return 1

    def cmd_expire(self, session, args):
        return self._set_deadline(session, args[0], _int(args[1]))

    def cmd_pexpire(self, session, args):
        return self._set_deadline(session, args[0], _int(args[1]) / 1000.0)

    def cmd_persist(self, session, args):
        if not self._alive(session, args[0]):
            return 0
        return int(self._expires[session.db].pop(args[0], None) is not None)

    def _remaining(self, session, key, scale):
        if not self._alive(session, key):
            return -2
        deadline = self._expires[session.db].get(key)
        if deadline is None:
            return -1
        return max(0, int(round((deadline - time.monotonic()) * scale)))

    def cmd_ttl(self, session, args):
        return self._remaining(session, args[0], 1)

    def cmd_pttl(self, session, args):
        return self._remaining(session, args[0], 1000)

    def cmd_rename(self, session, args):
        src, dst = args[0], args[1]
        if not self._alive(session, src):
            return ReplyError('ERR no such key')
        db = self._db(session)
        value = db.pop(src)
        deadline = self._expires[session.db].pop(src, None)
        self._delete(session, dst)
        db[dst] = value
        if deadline is not None:
            self._expires[session.db][dst] = deadline
        return OK

    def cmd_scan(self, session, args):
        cursor = _int(args[0])
        match, count, kind = None, 10, None
        i = 1
        while i < len(args):
            opt = args[i].upper()
            if opt == b'MATCH':
                match = args[i + 1]
            elif opt == b'COUNT':
                count = max(1, _int(args[i + 1]))
            elif opt == b'TYPE' and self.version >= (6, 0):
                kind = args[i + 1].lower()
            else:
                return ReplyError('ERR syntax error')
            i += 2
        # cursor = position in the sorted keyspace; expiry is checked only
        # for the keys of this window (not a full sweep per call)
        keys = sorted(self._dbs[session.db])
        window = keys[cursor:cursor + count]
        nxt = cursor + count if cursor + count < len(keys) else 0
        out = []
        types = {bytes: b'string', list: b'list', dict: b'hash', set: b'set'}
        for key in window:
            if match is not None and not glob_match(match, key):
                continue
            if not self._alive(session, key):
                continue
            if kind is not None and types[type(self._db(session)[key])] != kind:
                continue
            out.append(key)
        return [str(nxt).encode(), out]

    # -- strings -------------------------------------------------------------
    def cmd_get(self, session, args):
        return self._get(session, args[0], bytes)

    def cmd_set(self, session, args):
        key, value = args[0], args[1]
        ttl, nx, xx = None, False, False
        i = 2
        while i < len(args):
            opt = args[i].upper()
            if opt == b'EX':
                ttl = _int(args[i + 1])
                i += 1
            elif opt == b'PX':
                ttl = _int(args[i + 1]) / 1000.0
                i += 1
            elif opt == b'NX':
                nx = True
            elif opt == b'XX':
                xx = True
            i += 1
        exists = self._alive(session, key)
        if (nx and exists) or (xx and not exists):
            return None
        self._delete(session, key)
        self._db(session)[key] = value
        if ttl is not None:
            self._expires[session.db][key] = time.monotonic() + ttl
        return OK

    def cmd_setnx(self, session, args):
        if self._alive(session, args[0]):
            return 0
        self._db(session)[args[0]] = args[1]
        return 1

    def cmd_mget(self, session, args):
        out = []
        for key in args:
            value = self._alive(session, key) and self._db(session)[key]
            out.append(value if isinstance(value, bytes) else None)
        return out

    def cmd_mset(self, session, args):
        for key, value in zip(args[0::2], args[1::2]):
            self._delete(session, key)
            self._db(session)[key] = value
        return OK

    def cmd_incrby(self, session, args):
        current = self._get(session, args[0], bytes)
        number = _int(current if current is not None else 0) + _int(args[1])
        self._db(session)[args[0]] = str(number).encode()
        return number

    def cmd_incr(self, session, args):
        return self.cmd_incrby(session, [args[0], b'1'])

    def cmd_decrby(self, session, args):
        return self.cmd_incrby(session, [args[0], str(-_int(args[1])).encode()])

    def cmd_decr(self, session, args):
        return self.cmd_incrby(session, [args[0], b'-1'])

    # -- lists ---------------------------------------------------------------
    def cmd_lpush(self, session, args):
        lst = self._get_or_create(session, args[0], list)
        for value in args[1:]:
            lst.insert(0, value)
        return len(lst)

    def cmd_rpush(self, session, args):
        lst = self._get_or_create(session, args[0], list)
        lst.extend(args[1:])
        return len(lst)

    def _pop(self, session, args, left):
        lst = self._get(session, args[0], list)
        if len(args) > 1:
            count = _int(args[1])
            if lst is None:
                return NULL_ARRAY
            taken = []
            for _ in range(min(count, len(lst))):
                taken.append(lst.pop(0) if left else lst.pop())
            self._drop_if_empty(session, args[0], lst)
            return taken
        if not lst:
            return None
        value = lst.pop(0) if left else lst.pop()
        self._drop_if_empty(session, args[0], lst)
        return value

    def cmd_lpop(self, session, args):
        return self._pop(session, args, True)

    def cmd_rpop(self, session, args):
        return self._pop(session, args, False)

    def cmd_llen(self, session, args):
        lst = self._get(session, args[0], list)
        return len(lst) if lst else 0

    @staticmethod
    def _span(length, start, stop):
        if start < 0:
            start = max(0, length + start)
        if stop < 0:
            stop = length + stop
        return start, min(stop, length - 1)

    def cmd_lrange(self, session, args):
        lst = self._get(session, args[0], list) or []
        start, stop = self._span(len(lst), _int(args[1]), _int(args[2]))
        return lst[start:stop + 1] if start <= stop else []

    def cmd_lindex(self, session, args):
        lst = self._get(session, args[0], list) or []
        index = _int(args[1])
        try:
            return lst[index]
        except IndexError:
            return None

    def cmd_lset(self, session, args):
        lst = self._get(session, args[0], list)
        if lst is None:
            return ReplyError('ERR no such key')
        index = _int(args[1])
        try:
            lst[index] = args[2]
        except IndexError:
            return ReplyError('ERR index out of range')
        return OK

    def cmd_lrem(self, session, args):
        lst = self._get(session, args[0], list)
        if not lst:
            return 0
        count, value = _int(args[1]), args[2]
        removed = 0
        if count >= 0:
            i = 0
            while i < len(lst) and (count == 0 or removed < count):
                if lst[i] == value:
                    del lst[i]
                    removed += 1
                else:
                    i += 1
        else:
            i = len(lst) - 1
            while i >= 0 and removed < -count:
                if lst[i] == value:
                    del lst[i]
                    removed += 1
                i -= 1
        self._drop_if_empty(session, args[0], lst)
        return removed

    def cmd_ltrim(self, session, args):
        lst = self._get(session, args[0], list)
        if lst is None:
            return OK
        start, stop = self._span(len(lst), _int(args[1]), _int(args[2]))
        lst[:] = lst[start:stop + 1] if start <= stop else []
        self._drop_if_empty(session, args[0], lst)
        return OK

    def _move(self, session, src, dst, wherefrom, whereto):
        lst = self._get(session, src, list)
        if not lst:
            return None
        target = self._get(session, dst, list)  # WRONGTYPE check first
        value = lst.pop(0) if wherefrom == b'LEFT' else lst.pop()
        self._drop_if_empty(session, src, lst)
        if target is None:
            target = self._get_or_create(session, dst, list)
        if whereto == b'LEFT':
            target.insert(0, value)
        else:
            target.append(value)
        return value

    def cmd_lmove(self, session, args):
        return self._move(session, args[0], args[1], args[2].upper(),
                          args[3].upper())

    def cmd_rpoplpush(self, session, args):
        return self._move(session, args[0], args[1], b'RIGHT', b'LEFT')

    def _block(self, timeout, attempt):
        """Run ``attempt`` under the lock until it yields or time runs out."""
        deadline = None if timeout <= 0 else time.monotonic() + timeout
        with self._cond:
            while True:
                self.commands_processed += 1
                result = attempt()
                if result is not None:
                    self._cond.notify_all()
                    return result
                if deadline is None:
                    self._cond.wait(0.5)
                else:
                    remaining = deadline - time.monotonic()
                    if remaining <= 0:
                        return None
                    self._cond.wait(min(remaining, 0.5))

    def cmd_blmove(self, session, args):
        src, dst = args[0], args[1]
        frm, to = args[2].upper(), args[3].upper()
        timeout = self._timeout(args[4])
        return self._block(timeout,
                           lambda: self._move(session, src, dst, frm, to))

    def cmd_brpoplpush(self, session, args):
        timeout = self._timeout(args[2])
        return self._block(timeout, lambda: self._move(
            session, args[0], args[1], b'RIGHT', b'LEFT'))

    def _bpop(self, session, args, left):
        keys, timeout = args[:-1], self._timeout(args[-1])

        def attempt():
            for key in keys:
                lst = self._get(session, key, list)
                if lst:
                    value = lst.pop(0) if left else lst.pop()
                    self._drop_if_empty(session, key, lst)
                    return [key, value]
            return None
        result = self._block(timeout, attempt)
        return NULL_ARRAY if result is None else result

    def cmd_blpop(self, session, args):
        return self._bpop(session, args, True)

    def cmd_brpop(self, session, args):
        return self._bpop(session, args, False)

    # -- hashes --------------------------------------------------------------
    def cmd_hset(self, session, args):
        if len(args) < 3 or len(args) % 2 == 0:
            raise ValueError('arity')
        table = self._get_or_create(session, args[0], dict)
        added = 0
        for field, value in zip(args[1::2], args[2::2]):
            added += field not in table
            table[field] = value
        return added

    def cmd_hmset(self, session, args):
        self.cmd_hset(session, args)
        return OK

    def cmd_hsetnx(self, session, args):
        table = self._get_or_create(session, args[0], dict)
        if args[1] in table:
            return 0
        table[args[1]] = args[2]
        return 1

    def cmd_hget(self, session, args):
        table = self._get(session, args[0], dict) or {}
        return table.get(args[1])

    def cmd_hmget(self, session, args):
        table = self._get(session, args[0], dict) or {}
        return [table.get(f) for f in args[1:]]

    def cmd_hgetall(self, session, args):
        table = self._get(session, args[0], dict) or {}
        flat = []
        for field, value in table.items():
            flat += [field, value]
        return flat

    def cmd_hdel(self, session, args):
        table = self._get(session, args[0], dict)
        if not table:
            return 0
        removed = sum(1 for f in args[1:] if table.pop(f, None) is not None)
        self._drop_if_empty(session, args[0], table)
        return removed

    def cmd_hlen(self, session, args):
        return len(self._get(session, args[0], dict) or {})

    def cmd_hexists(self, session, args):
        return int(args[1] in (self._get(session, args[0], dict) or {}))

    def cmd_hincrby(self, session, args):
        table = self._get_or_create(session, args[0], dict)
        number = _int(table.get(args[1], b'0')) + _int(args[2])
        table[args[1]] = str(number).encode()
        return number

    def cmd_hkeys(self, session, args):
        return list((self._get(session, args[0], dict) or {}).keys())

    def cmd_hvals(self, session, args):
        return list((self._get(session, args[0], dict) or {}).values())

    # -- sets ----------------------------------------------------------------
    def cmd_sadd(self, session, args):
        members = self._get_or_create(session, args[0], set)
        before = len(members)
        members.update(args[1:])
        return len(members) - before

    def cmd_srem(self, session, args):
        members = self._get(session, args[0], set)
        if not members:
            return 0
        removed = sum(1 for m in args[1:] if m in members
                      and not members.discard(m))
        self._drop_if_empty(session, args[0], members)
        return removed

    def cmd_smembers(self, session, args):
        return sorted(self._get(session, args[0], set) or ())

    def cmd_scard(self, session, args):
        return len(self._get(session, args[0], set) or ())

    def cmd_sismember(self, session, args):
        return int(args[1] in (self._get(session, args[0], set) or ()))

    # -- pub/sub, scripting --------------------------------------------------
    def cmd_publish(self, session, args):
        return 0

    def cmd_eval(self, session, args):
        return ReplyError('ERR scripting is not supported by this engine')

    cmd_evalsha = cmd_eval

    def cmd_script(self, session, args):
        if args and args[0].upper() == b'KILL':
            return ReplyError('NOTBUSY No scripts in execution right now.')
        return ReplyError('ERR scripting is not supported by this engine')

    # -- sentinel personality ------------------------------------------------
    @staticmethod
    def _flat_state(name, ip, port, flags):
        return [b'name', _b(name), b'ip', _b(ip), b'port', _b(port),
                b'flags', _b(flags), b'role-reported', b'master'
                if flags == 'master' else b'slave']

    def cmd_sentinel(self, session, args):
        if not self.sentinel_masters:
            return ReplyError("ERR unknown command 'sentinel', with args "
                              "beginning with: ")
        sub = args[0].upper()
        if sub == b'MASTERS':
            return [self._flat_state(name, m['ip'], m['port'], 'master')
                    for name, m in self.sentinel_masters.items()]
        if sub in (b'SLAVES', b'REPLICAS'):
            master = self.sentinel_masters.get(args[1].decode('utf-8'))
            if master is None:
                return ReplyError('ERR No such master with that name')
            return [self._flat_state('%s:%s' % (ip, port), ip, port, 'slave')
                    for ip, port in master.get('replicas', [])]
        if sub == b'GET-MASTER-ADDR-BY-NAME':
            master = self.sentinel_masters.get(args[1].decode('utf-8'))
            if master is None:
                return None
            return [_b(master['ip']), _b(master['port'])]
        return ReplyError('ERR Unknown sentinel subcommand')


class LoopbackConnection(object):
    """A :class:`~kiosk_autoscaler_amd.redisq.Connection` stand-in that
    executes against an engine, round-tripping replies through RESP."""

    def __init__(self, engine, decode_responses=True, encoding='utf-8'):
        self.engine = engine
        self.session = Session()
        self.decode_responses = decode_responses
        self.encoding = encoding
        self._parser = RespParser(decode=decode_responses, encoding=encoding)
        self.connected = True

    def connect(self):
        self.connected = True

    def disconnect(self):
        self.connected = False
        self.session = Session()
        self._parser = RespParser(decode=self.decode_responses,
                                  encoding=self.encoding)

    def _run(self, args):
        try:
            reply = self.engine.execute(self.session, list(args))
        except DropConnection as dropped:
            self.disconnect()
            raise exceptions.ConnectionError(
                'Connection reset by peer (injected on %s)' % dropped)
        self._parser.feed(encode_reply(reply))

    def send_command(self, *args):
        self._run(args)

    def send_commands(self, commands):
        for cmd in commands:
            self._run(cmd)

    def read_response(self, timeout=None):
        from ..redisq.connection import _materialize_errors
        reply = self._parser.gets()
        if reply is NOT_READY:
            raise exceptions.ConnectionError('no pending reply')
        return _materialize_errors(reply)


class LoopbackPool(object):
    """Connection pool handing out :class:`LoopbackConnection` objects."""

    def __init__(self, engine, decode_responses=True, encoding='utf-8'):
        self.engine = engine
        self.decode_responses = decode_responses
        self.encoding = encoding
        self._local = threading.local()

    def get_connection(self):
        # one connection per thread keeps MULTI/SELECT state per caller
        conn = getattr(self._local, 'conn', None)
        if conn is None:
            conn = LoopbackConnection(self.engine, self.decode_responses,
                                      self.encoding)
            self._local.conn = conn
        if not conn.connected:
            conn.connect()
        return conn

    def release(self, conn):
        pass

    def disconnect(self):
        conn = getattr(self._local, 'conn', None)
        if conn is not None:
            conn.disconnect()


class FakeRedis(Redis):
    """The framework's Redis client bound to an in-process engine.

    ``FakeRedis()`` makes a private engine; pass ``engine=`` to share one
    keyspace between several clients (how the sentinel fakes model a
    master with replicas)."""

    def __init__(self, engine=None, decode_responses=True, encoding='utf-8',
                 **_ignored):
        self.engine = engine if engine is not None else RedisEngine()
        Redis.__init__(self, connection_pool=LoopbackPool(
            self.engine, decode_responses, encoding))


FakeStrictRedis = FakeRedis
