"""Worker fault injection ("kill -9 a worker, drop the Redis
socket, return BUSY, hang a kernel").

The reference injects faults only inside its unit tests
(``autoscaler/redis_test.py:55-68``, ``autoscaler/autoscaler_test.py:45-46``).
Here the same failure classes can be provoked in real worker processes, so
the manager's detection/recovery path (waitpid reaping, watchdog, requeue,
restart backoff, fence abort) is exercised end to end.  Redis-side faults
(connection drop, BUSY, error replies) live in the fake engine
(:meth:`kiosk_autoscaler_amd.fakes.engine.RedisEngine.inject_fault`).

Spec (env ``KIOSK_FAULTS``, comma separated)::

    crash_key=N        exit(86) just before serving the N-th key (1-based)
    hang_key=N[:MS]    stall the N-th key for MS ms (default 30000): on the
                       HIP engine a bounded spinning kernel on the serving
                       stream (a real stuck GPU job), on the CPU mock a sleep
    slow_start=MS      sleep MS ms between "weights ready" and READY
    fail_start         raise during start-up (exit code 3, no READY)
    drop_redis_key=N   close the worker's Redis connections before key N
                       (the retrying client must reconnect transparently)
    freeze_agent=N[:MS]  before key N, freeze the process's node-fence agent
                       thread for MS ms (default 20000) at its next fence:
                       a serving rank that stops answering, the process and
                       its key otherwise healthy

Each fault fires at most once per run of the whole stack: the first worker
to reach it claims ``kiosk:fault:<name>`` with ``SET NX`` (TTL 1 h), so the
replacement worker the manager starts afterwards runs clean and the test
can observe recovery.  Without a Redis client every fault fires once per
process.
"""
import logging
import os
import time

logger = logging.getLogger('Faults')

CLAIM_KEY = 'kiosk:fault:{name}'
CRASH_CODE = 86
KINDS = ('crash_key', 'hang_key', 'slow_start', 'fail_start',
         'drop_redis_key', 'freeze_agent')


class InjectedFault(RuntimeError):
    pass


def parse(spec):
    """``'hang_key=2:500,fail_start'`` -> ``{'hang_key': (2, 500.0),
    'fail_start': ()}``."""
    faults = {}
    for part in (spec or '').split(','):
        part = part.strip()
        if not part:
            continue
        name, _, value = part.partition('=')
        name = name.strip()
        if name not in KINDS:
            raise ValueError('unknown fault %r (known: %s)' % (
                name, ', '.join(KINDS)))
        args = tuple(float(v) for v in value.split(':') if v.strip()) \
            if value else ()
        if name in ('crash_key', 'hang_key', 'drop_redis_key',
                    'freeze_agent') and not args:
            raise ValueError('%s needs a key index' % name)
        if name == 'slow_start' and not args:
            raise ValueError('slow_start needs milliseconds')
        faults[name] = args
    return faults


class FaultPlan(object):
    def __init__(self, faults, redis=None, owner=''):
        self.faults = dict(faults)
        self.redis = redis
        self.owner = owner
        self.fired = []

    @classmethod
    def from_env(cls, env=None, redis=None, owner=''):
        env = os.environ if env is None else env
        return cls(parse(env.get('KIOSK_FAULTS', '')), redis, owner)

    def __bool__(self):
        return bool(self.faults)

    def _claim(self, name):
        if name in self.fired:
            return False
        if self.redis is not None:
            try:
                if not self.redis.set(CLAIM_KEY.format(name=name),
                                      self.owner or str(os.getpid()),
                                      nx=True, ex=3600):
                    return False
            except Exception as err:  # pylint: disable=broad-except
                logger.warning('fault claim for %s failed: %s', name, err)
                return False
        self.fired.append(name)
        logger.warning('injecting fault %s in %s', name, self.owner)
        return True

    def at_start(self):
        """Between 'weights ready' and READY."""
        if 'fail_start' in self.faults and self._claim('fail_start'):
            raise InjectedFault('injected start-up failure')
        if 'slow_start' in self.faults and self._claim('slow_start'):
            time.sleep(self.faults['slow_start'][0] / 1e3)

    def before_key(self, index, engine=None, redis=None, agent=None):
        """``index`` is 1-based over this worker's served keys."""
        f = self.faults
        if 'freeze_agent' in f and agent is not None and \
                index == int(f['freeze_agent'][0]) and \
                self._claim('freeze_agent'):
            args = f['freeze_agent']
            agent.freeze_next_fence(args[1] if len(args) > 1 else 20000.0)
        if 'drop_redis_key' in f and index == int(f['drop_redis_key'][0]) \
                and self._claim('drop_redis_key'):
            _drop_connections(redis)
        if 'crash_key' in f and index == int(f['crash_key'][0]) \
                and self._claim('crash_key'):
            os._exit(CRASH_CODE)
        if 'hang_key' in f and index == int(f['hang_key'][0]) \
                and self._claim('hang_key'):
            args = f['hang_key']
            ms = args[1] if len(args) > 1 else 30000.0
            if engine is not None and hasattr(engine, 'spin'):
                engine.spin(ms)
            else:
                time.sleep(ms / 1e3)


def _drop_connections(redis):
    """Close every pooled socket of a (failover) client."""
    if redis is None:
        return
    clients = []
    for attr in ('_redis_master', '_redis_slaves'):
        value = getattr(redis, '__dict__', {}).get(attr)
        if isinstance(value, list):
            clients.extend(value)
        elif value is not None:
            clients.append(value)
    if not clients:
        clients = [redis]
    for client in clients:
        pool = getattr(client, 'connection_pool', None)
        if pool is not None:
            pool.disconnect()
