"""Sentinel-aware, retrying Redis proxy (component C1-C4 of SURVEY §2.1).

Behavioural contract kept from the reference (``autoscaler/redis.py``):

* C1 routing (``redis.py:38-122, 170-173``): commands in
  :data:`REDIS_READONLY_COMMANDS` go to a uniformly random replica, every other
  command to the master.  ``scan_iter`` is deliberately *not* read-only (only
  ``scan`` is), so the tally's SCAN walks the master while its LLEN hits a
  replica -- characterised in SURVEY §2.1 C1.
* C2 construction (``redis.py:125-133``): the configured host is treated as
  the sentinel; master and replica set start as that single client; then C3.
  A connection error during construction propagates (crash-only startup).
* C3 discovery (``redis.py:135-155``): ``SENTINEL MASTERS`` then, per master
  set, ``SENTINEL SLAVES``; the last set wins.  A ``ResponseError`` (plain
  Redis, "unknown command") keeps the single client and logs a warning.
* C4 retry (``redis.py:163-202``): ``ConnectionError`` -> rediscover, warn,
  sleep ``backoff`` and retry forever (but an error raised by the
  rediscovery itself escapes); ``ResponseError`` mentioning both ``BUSY`` and
  ``SCRIPT KILL`` -> warn, sleep, retry; any other ``ResponseError`` is
  re-raised; anything else (including ``AttributeError`` for an unknown
  command) is logged at ERROR and re-raised.  Generators are returned
  unconsumed, so iteration errors are outside the retry.

Framework additions (all opt-in, defaults keep the contract above):
``max_retries`` bounds the ConnectionError loop and ``backoff_cap`` /
``backoff_factor`` turn the fixed sleep into capped exponential backoff.
"""
import logging
import random
import time

from . import exceptions
from .client import StrictRedis

# Read-only command table (C1).  Grouped by data type for readability; the
# set is the same 83 names the reference routes to replicas.
_READONLY_BY_GROUP = {
    'connection': 'auth echo ping select readonly readwrite asking',
    'server': 'client command dbsize info lastsave slowlog time '
              'pfselftest wait',
    'transactions': 'discard multi unwatch watch',
    'pubsub': 'publish subscribe unsubscribe psubscribe punsubscribe pubsub',
    'scripting': 'script',
    'keys': 'dump exists keys object pttl randomkey scan ttl type',
    'strings': 'bitcount bitpos get getbit getrange mget strlen substr',
    'lists': 'lindex llen lrange',
    'hashes': 'hexists hget hgetall hkeys hlen hmget hscan hstrlen hvals',
    'sets': 'scard sdiff sinter sismember smembers srandmember sscan sunion',
    'sorted_sets': 'zcard zcount zlexcount zrange zrangebylex zrangebyscore '
                   'zrank zrevrange zrevrangebylex zrevrangebyscore zrevrank '
                   'zscan zscore',
    'geo': 'geodist geohash geopos georadius georadiusbymember',
    'hyperloglog': 'pfcount',
}

REDIS_READONLY_COMMANDS = frozenset(
    name for group in _READONLY_BY_GROUP.values() for name in group.split())


class RedisClient(object):
    """Fault-tolerant proxy exposing every client command as an attribute.

    Args:
        host: sentinel (or plain Redis) host.
        port: its port.
        backoff: seconds to sleep between retries (``REDIS_INTERVAL``).
        max_retries: ``None`` (reference behaviour: retry forever) or a bound
            on consecutive ConnectionError retries per call.
        backoff_factor / backoff_cap: exponential growth of the sleep; the
            default factor 1 keeps the reference's fixed backoff.
    """

    def __init__(self, host, port, backoff=1, max_retries=None,
                 backoff_factor=1.0, backoff_cap=None):
        self.logger = logging.getLogger(str(self.__class__.__name__))
        self.backoff = backoff
        self.max_retries = max_retries
        self.backoff_factor = float(backoff_factor)
        self.backoff_cap = backoff_cap
        self._sentinel = self._get_redis_client(host=host, port=port)
        self._redis_master = self._sentinel
        self._redis_slaves = [self._sentinel]
        self._update_masters_and_slaves()

    @classmethod
    def _get_redis_client(cls, host, port):
        return StrictRedis(host=host, port=port, decode_responses=True,
                           charset='utf-8')

    def _update_masters_and_slaves(self):
        """C3: refresh master/replica clients from the sentinel."""
        try:
            masters = self._sentinel.sentinel_masters()
            for set_name, state in masters.items():
                master = self._get_redis_client(state['ip'], state['port'])
                replicas = [
                    self._get_redis_client(r['ip'], r['port'])
                    for r in self._sentinel.sentinel_slaves(set_name)]
                # the last master set wins, as in the reference
                self._redis_master = master
                self._redis_slaves = replicas
        except exceptions.ResponseError as err:
            self.logger.warning('Encountered Error: %s. Using sentinel as '
                                'primary redis client.', err)

    def _node_for(self, command):
        if command in REDIS_READONLY_COMMANDS and self._redis_slaves:
            return random.choice(self._redis_slaves)
        return self._redis_master

    def _sleep_for(self, attempt):
        delay = self.backoff * (self.backoff_factor ** attempt)
        if self.backoff_cap is not None:
            delay = min(delay, self.backoff_cap)
        return delay

    def __getattr__(self, name):
        if name.startswith('_'):
            raise AttributeError(name)

        def call_with_retry(*args, **kwargs):
            shown = ' '.join(str(v) for v in list(args) + list(kwargs.values()))
            attempt = 0
            while True:
                try:
                    command = getattr(self._node_for(name), name)
                    return command(*args, **kwargs)
                except exceptions.ConnectionError as err:
                    # an error from rediscovery itself escapes (C4)
                    self._update_masters_and_slaves()
                    if (self.max_retries is not None
                            and attempt >= self.max_retries):
                        raise
                    delay = self._sleep_for(attempt)
                    self.logger.warning(
                        'Encountered %s: %s when calling `%s %s`. '
                        'Retrying in %s seconds.', type(err).__name__, err,
                        name.upper(), shown, delay)
                    time.sleep(delay)
                    attempt += 1
                except exceptions.ResponseError as err:
                    text = str(err)
                    if 'BUSY' not in text or 'SCRIPT KILL' not in text:
                        raise
                    self.logger.warning(
                        'Encountered %s: %s when calling `%s %s`. '
                        'Retrying in %s seconds.', type(err).__name__, err,
                        name.upper(), shown, self.backoff)
                    time.sleep(self.backoff)
                except Exception as err:
                    self.logger.error('Unexpected %s: %s when calling `%s %s`.',
                                      type(err).__name__, err, name.upper(),
                                      shown)
                    raise

        call_with_retry.__name__ = name
        return call_with_retry
