"""Sentinel-mode and fault-injecting fakes.

Models, without a network, what the reference's ``WrappedFakeStrictRedis``
models (``autoscaler/redis_test.py:41-68``): a sentinel that reports one
master set with 2-5 replicas, all sharing one keyspace, plus one-shot
``ConnectionError`` / ``BUSY`` fault injectors.
"""
import random

from ..redisq import exceptions
from .engine import BUSY_MESSAGE, FakeRedis, RedisEngine


class SentinelCluster(object):
    """A sentinel + master + replicas topology held in-process.

    ``factory(host, port)`` returns a client for any address: the sentinel
    address gets the sentinel personality, every other address reads and
    writes the shared data engine (instant replication).  Plug it into
    :class:`~kiosk_autoscaler_amd.redisq.RedisClient` by patching
    ``RedisClient._get_redis_client``.
    """

    def __init__(self, sentinel=('sentinel', 26379), master_name='mymaster',
                 master=('master', 6379), replicas=None, seed=None):
        rng = random.Random(seed)
        if replicas is None:
            replicas = [('slave', 6379)] * rng.randint(2, 5)
        self.sentinel_addr = tuple(sentinel)
        self.data = RedisEngine()
        self.sentinel = RedisEngine(sentinel_masters={
            master_name: {'ip': master[0], 'port': master[1],
                          'replicas': list(replicas)}})
        self.created = []

    def factory(self, host, port):
        if (host, int(port)) == (self.sentinel_addr[0],
                                 int(self.sentinel_addr[1])):
            client = FakeRedis(engine=self.sentinel)
        else:
            client = FakeRedis(engine=self.data)
        client.address = (host, int(port))
        self.created.append(client)
        return client


class FlakyRedis(FakeRedis):
    """FakeRedis with the reference test's one-shot fault methods.

    ``busy_error`` raises a BUSY/SCRIPT KILL ``ResponseError`` once,
    ``connect_error`` raises ``ConnectionError`` once, ``fail`` always raises
    a plain ``ResponseError`` (``autoscaler/redis_test.py:55-68``)."""

    def __init__(self, engine=None, should_fail=False, **kwargs):
        FakeRedis.__init__(self, engine=engine, **kwargs)
        self.should_fail = should_fail

    def sentinel_masters(self):
        return {'mymaster': {'ip': 'master', 'port': 6379}}

    def sentinel_slaves(self, service_name):
        return [{'ip': 'slave', 'port': 6379}
                for _ in range(random.randint(2, 5))]

    def busy_error(self, *_, **__):
        if self.should_fail:
            self.should_fail = False
            raise exceptions.ResponseError(BUSY_MESSAGE)
        return True

    def connect_error(self, *_, **__):
        if self.should_fail:
            self.should_fail = False
            raise exceptions.ConnectionError('thrown on purpose')
        return True

    def fail(self, *_, **__):
        raise exceptions.ResponseError('thrown on purpose')
