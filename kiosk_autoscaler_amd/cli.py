"""Process entry point: env config -> logging -> clients -> reconcile loop.

Behaviour of the reference's ``scale.py`` (C16-C18, ``scale.py:69-106``):

* logging as :func:`~kiosk_autoscaler_amd.utils.logs.initialize_logger`;
* a sentinel-aware :class:`RedisClient` built from ``REDIS_HOST/PORT`` with
  ``REDIS_INTERVAL`` backoff -- a connection error here crashes startup;
* ``RESOURCE_NAME`` is required (missing -> ``UndefinedValueError``);
* ``while True: scale(); gc.collect(); sleep(INTERVAL)`` -- the period is
  tick time + ``INTERVAL`` (``FIXED_RATE=1`` makes it exactly ``INTERVAL``);
* any exception -> CRITICAL ``Fatal Error: <type>: <msg>`` and exit 1.

The actuator is the node-local GPU manager: embedded in this process by
default (its workers are drained when the process exits) or a separate
daemon (``GPUMGR=unix:PATH``; workers then survive autoscaler restarts).
"""
import gc
import logging
import signal
import sys
import time

from . import gpumgr
from .autoscaler import Autoscaler
from .config import Settings
from .redisq import RedisClient
from .utils.events import EventLog
from .utils.logs import flush_deferred, initialize_logger


class _Terminate(Exception):
    pass


def _on_sigterm(signum, frame):
    raise _Terminate('signal %d' % signum)


def build(settings=None, redis_client=None, actuator=None, events=None):
    """Construct (client, scaler, manager) exactly as ``main`` would."""
    settings = settings or Settings()
    if redis_client is None:
        redis_client = RedisClient(host=settings.REDIS_HOST,
                                   port=settings.REDIS_PORT,
                                   backoff=settings.REDIS_INTERVAL)
    if events is None:
        if settings.EVENT_LOG == 'redis':
            events = EventLog(redis_client=redis_client, source='autoscaler')
        else:
            events = EventLog(path=settings.EVENT_LOG or None,
                              source='autoscaler')
    manager = None
    if actuator is None:
        if settings.GPUMGR.startswith('unix:') or \
                settings.GPUMGR.startswith('k8s'):
            # with k8s the Deployment/Job already exists in the cluster; a
            # shared manager daemon learns this autoscaler's resource here
            # (an invalid RESOURCE_TYPE stays fatal at the first tick, as in
            # the reference)
            actuator = gpumgr.connect(settings.GPUMGR)
            if settings.GPUMGR.startswith('unix:') and \
                    settings.RESOURCE_TYPE in ('deployment', 'job'):
                actuator.register(settings.RESOURCE_TYPE,
                                  settings.RESOURCE_NAMESPACE,
                                  settings.RESOURCE_NAME,
                                  gpumgr.template_for(settings))
        else:
            manager = gpumgr.build_manager(settings, redis_client=redis_client,
                                           events=events)
            if 0 < len(manager.slots) < settings.MAX_PODS:
                # one worker per GPU, so MAX_PODS beyond the
                # node's GPUs could only ever be pending
                logging.getLogger('autoscaler').warning(
                    'MAX_PODS=%d exceeds the %d GPU slots of this node; '
                    'clamping to %d.', settings.MAX_PODS, len(manager.slots),
                    len(manager.slots))
                settings.MAX_PODS = len(manager.slots)
            manager.start()
            gpumgr.set_embedded(manager)
            actuator = manager
    if settings.METRICS_PORT:
        from .utils import metrics
        metrics.attach(events, settings.METRICS_PORT, manager=manager,
                       addr=settings.METRICS_ADDR)
    scaler = Autoscaler(redis_client=redis_client, queues=settings.QUEUES,
                        queue_delim=settings.QUEUE_DELIMITER,
                        actuator=actuator, policy=settings.policy,
                        scale_down_delay=settings.SCALE_DOWN_DELAY,
                        zero_delay=getattr(settings, 'SCALE_TO_ZERO_DELAY',
                                           0.0),
                        events=events, tally=settings.TALLY_MODE)
    return redis_client, scaler, manager


def run_loop(scaler, settings, max_ticks=None, sleep=time.sleep,
             clock=time.monotonic):
    """The reconcile loop; returns after ``max_ticks`` (tests) or never."""
    ticks = 0
    next_tick = clock()
    tick_key = getattr(settings, 'TICK_KEY', '')
    while max_ticks is None or ticks < max_ticks:
        started = time.monotonic_ns()
        scaler.scale(namespace=settings.RESOURCE_NAMESPACE,
                     resource_type=settings.RESOURCE_TYPE,
                     name=settings.RESOURCE_NAME,
                     min_pods=settings.MIN_PODS,
                     max_pods=settings.MAX_PODS,
                     keys_per_pod=settings.KEYS_PER_POD)
        gc.collect()
        if tick_key:
            # observability hook for the benchmark's phase control
            scaler.redis_client.set(tick_key, '%d %d %d' % (
                started, time.monotonic_ns(), ticks))
        # the tick's log records are written now, after its decision
        flush_deferred()
        ticks += 1
        if max_ticks is not None and ticks >= max_ticks:
            break
        interval = settings.INTERVAL
        idle = getattr(settings, 'IDLE_INTERVAL', 0.0)
        if idle and 0 < idle < interval and scaler.last_decision == 0:
            # opt-in fast path while scaled to zero: a cold start waits for
            # at most IDLE_INTERVAL instead of INTERVAL (not the reference's
            # semantics; reported separately in the benchmarks)
            interval = idle
        # an embedded manager wakes a parked pool just ahead of the tick
        # that will scale for a new key (POOL_WAKE_LEAD_S)
        note = getattr(scaler.actuator, 'note_next_tick', None)
        if settings.FIXED_RATE:
            next_tick += interval
            if callable(note):
                note(time.monotonic() + max(0.0, next_tick - clock()))
            sleep(max(0.0, next_tick - clock()))
        else:
            if callable(note):
                note(time.monotonic() + interval)
            sleep(interval)
    return ticks


def main(argv=None):
    del argv
    settings = Settings()   # missing RESOURCE_NAME raises here (fatal)
    initialize_logger(debug_mode=settings.DEBUG, log_file=settings.LOG_FILE)
    _logger = logging.getLogger(__file__)
    from .config import removed_knobs
    for name, hint in removed_knobs():
        _logger.warning('%s is set but no longer a setting of its own: %s.',
                        name, hint)
    signal.signal(signal.SIGTERM, _on_sigterm)
    manager = None
    try:
        _, scaler, manager = build(settings)
        run_loop(scaler, settings)
    except (KeyboardInterrupt, _Terminate) as err:
        _logger.info('Shutting down (%s).', err or 'interrupt')
        code = 0
    except Exception as err:  # pylint: disable=broad-except
        _logger.critical('Fatal Error: %s: %s', type(err).__name__, err)
        code = 1
    else:
        code = 0
    finally:
        if manager is not None:
            manager.stop()
    sys.exit(code)


if __name__ == '__main__':
    main()
