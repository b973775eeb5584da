"""The reconcile core: tally -> observe -> decide -> actuate (C5-C14).

Reference: ``autoscaler/autoscaler.py``.  The public method names and
argument orders match the reference so code written against it keeps
working; the Kubernetes client layer (C7-C9) is replaced by an *actuator*
with the same four calls -- by default the node-local GPU manager
(:mod:`kiosk_autoscaler_amd.gpumgr`), which launches / reaps PyTorch-ROCm
worker processes pinned to MI355X GPUs instead of patching a Deployment.

Behaviour kept:

* C6 tally: ``LLEN q`` + number of keys matching ``processing-q:*`` (SCAN,
  COUNT 1000), logged at INFO as ``In-progress or new redis keys``.
* C10 observe: unknown type -> ``ValueError``; missing resource -> 0;
  ``None`` -> 0; value ``int()``-cast; ``only_running`` reads READY workers.
* C11-C14 decide: :mod:`kiosk_autoscaler_amd.policy` (``reference`` default).
* C13 actuate: no call when ``desired == current`` (returns ``None``);
  otherwise patch and return ``True``.
* C14: only the actuator error raised by ``scale_resource`` is swallowed
  (WARNING); errors from tally/observe propagate (crash-only main loop).
"""
import logging
import timeit

from . import policy as policies
from .gpumgr.resources import ActuatorError
from .utils.events import NULL as NULL_EVENTS, now_ns
from .utils.keys import worker_of


class Autoscaler(object):
    """Read Redis and scale GPU worker processes when required.

    Reference: ``autoscaler/autoscaler.py:37-58`` (class, constructor).

    Args:
        redis_client: Redis client (``RedisClient`` proxy, ``Redis`` or fake).
        queues: delimiter-joined queue names.
        queue_delim: delimiter for ``queues``.
        actuator: object with ``list_namespaced_{deployment,job}`` and
            ``patch_namespaced_{deployment,job}``; defaults to a lazily
            created embedded GPU manager (:meth:`get_actuator`).
        policy: ``'reference'`` (bit-compatible) or ``'strict'``.
        scale_down_delay: seconds a lower target must persist before a
            scale-down is applied (``strict`` hysteresis; 0 = immediate).
        zero_delay: seconds a target of zero must persist before the last
            workers are scaled away (``strict``'s default hysteresis: a
            transient empty queue mid-burst would otherwise make the next
            key pay a cold start; scale-downs that keep workers are
            immediate).
        events: optional :class:`~kiosk_autoscaler_amd.utils.EventLog`.
        tally: ``'reference'`` (``LLEN`` on a replica, then a ``SCAN`` of
            the master: two non-atomic reads, SURVEY §5.2, so an item a
            worker moves in between can be counted twice or missed) or
            ``'atomic'`` (``LLEN`` + ``KEYS processing-q:*`` in one
            ``MULTI``/``EXEC`` on the master: one consistent snapshot).
    """

    def __init__(self, redis_client, queues='predict', queue_delim=',',
                 actuator=None, policy='reference', scale_down_delay=0.0,
                 events=None, clock=timeit.default_timer,
                 tally='reference', zero_delay=0.0):
        self.redis_keys = {q: 0 for q in queues.split(queue_delim)}
        self.in_progress = {q: 0 for q in self.redis_keys}
        # distinct workers holding processing keys (a batched worker holds
        # one key per slot: processing-q:<id>, processing-q:<id>.1, ...)
        self.busy_workers = set()
        self.redis_client = redis_client
        self.logger = logging.getLogger(str(self.__class__.__name__))
        self.managed_resource_types = {'deployment', 'job'}
        self.actuator = actuator
        if policy not in policies.POLICIES:
            raise ValueError('unknown policy %r' % policy)
        self.policy = policy
        self.scale_down_delay = float(scale_down_delay)
        self.zero_delay = float(zero_delay)
        self.events = events if events is not None else NULL_EVENTS
        self._clock = clock
        self._lower_since = None
        self.last_decision = None
        if tally not in ('reference', 'atomic'):
            raise ValueError('unknown tally mode %r' % tally)
        self.tally = tally

    # -- C6 ------------------------------------------------------------------
    def tally_queues(self):
        """Update ``redis_keys[q] = LLEN q + #keys('processing-q:*')``.

        Reference: ``autoscaler/autoscaler.py:60-77``."""
        start = self._clock()
        busy = set()
        for queue in self.redis_keys:
            self.logger.debug('Tallying items in queue `%s`.', queue)
            pattern = 'processing-{}:*'.format(queue)
            counted = None
            if self.tally == 'atomic':
                counted = self._tally_atomic(queue, pattern)
            if counted is None:
                waiting = self.redis_client.llen(queue)
                keys = list(self.redis_client.scan_iter(match=pattern,
                                                        count=1000))
            else:
                waiting, keys = counted
            running = len(keys)
            busy.update(worker_of(k) for k in keys)
            self.in_progress[queue] = running
            self.redis_keys[queue] = waiting + running
        self.busy_workers = busy
        self.logger.debug('Finished tallying redis keys in %s seconds.',
                          self._clock() - start)
        self.logger.info('In-progress or new redis keys: %s', self.redis_keys)
        return dict(self.redis_keys)

    def _tally_atomic(self, queue, pattern):
        """``(LLEN, #processing keys)`` from one MULTI/EXEC on the master, or
        ``None`` on a connection error (the caller falls back to the
        retrying reference path, so a failover still heals itself)."""
        from .redisq.exceptions import ConnectionError as RedisConnError
        try:
            pipe = self.redis_client.pipeline(transaction=True)
            pipe.llen(queue)
            pipe.keys(pattern)
            waiting, keys = pipe.execute()
        except RedisConnError as err:
            self.logger.warning('atomic tally of `%s` failed (%s); using '
                                'LLEN + SCAN', queue, err)
            return None
        return int(waiting), list(keys)

    # -- C7-C9: actuator access ------------------------------------------------
    def get_actuator(self):
        """The ``get_apps_v1_client``/``get_batch_v1_client`` analog
        (``autoscaler/autoscaler.py:79-87``)."""
        if self.actuator is None:
            from .gpumgr import connect
            self.actuator = connect()
        return self.actuator

    def _timed(self, what, func, *args):
        started = self._clock()
        try:
            result = func(*args)
        except ActuatorError as err:
            self.logger.error('%s when calling `%s`: %s',
                              type(err).__name__, what, err)
            raise
        self.logger.debug('%s finished in %s seconds.', what,
                          self._clock() - started)
        return result

    def list_namespaced_deployment(self, namespace):
        """Reference: ``autoscaler/autoscaler.py:89-104``."""
        items = self._timed('list_namespaced_deployment',
                            self.get_actuator().list_namespaced_deployment,
                            namespace).items
        self.logger.debug('Found %s deployments in namespace `%s`: %s',
                          len(items), namespace,
                          [d.metadata.name for d in items])
        return items

    def list_namespaced_job(self, namespace):
        """Reference: ``autoscaler/autoscaler.py:106-119``."""
        items = self._timed('list_namespaced_job',
                            self.get_actuator().list_namespaced_job,
                            namespace).items
        self.logger.debug('Found %s jobs in namespace `%s`.', len(items),
                          namespace)
        return items

    def patch_namespaced_deployment(self, name, namespace, body):
        """Reference: ``autoscaler/autoscaler.py:121-135``."""
        return self._timed('patch_namespaced_deployment',
                           self.get_actuator().patch_namespaced_deployment,
                           name, namespace, body)

    def patch_namespaced_job(self, name, namespace, body):
        """Reference: ``autoscaler/autoscaler.py:137-151``."""
        return self._timed('patch_namespaced_job',
                           self.get_actuator().patch_namespaced_job,
                           name, namespace, body)

    # -- C10 -----------------------------------------------------------------
    def _check_type(self, resource_type):
        if resource_type not in self.managed_resource_types:
            raise ValueError('`resource_type` must be one of {}. Got {}.'.format(
                self.managed_resource_types, resource_type))

    def get_current_pods(self, namespace, resource_type, name,
                         only_running=False):
        """Declared worker count (or READY count with ``only_running``).

        Reference: ``autoscaler/autoscaler.py:153-195``."""
        self._check_type(resource_type)
        if resource_type == 'deployment':
            items = self.list_namespaced_deployment(namespace)
        else:
            items = self.list_namespaced_job(namespace)
        count = 0
        for item in items:
            if item.metadata.name != name:
                continue
            if resource_type == 'job':
                count = item.spec.parallelism
            elif only_running:
                count = item.status.available_replicas
            else:
                count = item.spec.replicas
            self.logger.debug('%s %s has %s pods', resource_type, name, count)
            break
        return int(count or 0)

    # -- C11 / C12 -------------------------------------------------------------
    def clip_pod_count(self, desired_pods, min_pods, max_pods, current_pods):
        """Reference: ``autoscaler/autoscaler.py:197-213``."""
        clipped = policies.clip_pod_count(desired_pods, min_pods, max_pods,
                                          current_pods)
        if clipped != desired_pods:
            self.logger.debug('Clipped pods from %s to %s', desired_pods,
                              clipped)
        return clipped

    def get_desired_pods(self, key, keys_per_pod, min_pods, max_pods,
                         current_pods):
        """Reference: ``autoscaler/autoscaler.py:215-219`` (floor)."""
        return self.clip_pod_count(self.redis_keys[key] // keys_per_pod,
                                   min_pods, max_pods, current_pods)

    # -- C13 -----------------------------------------------------------------
    def scale_resource(self, desired_pods, current_pods, resource_type,
                       namespace, name):
        """Reference: ``autoscaler/autoscaler.py:221-242``."""
        if resource_type not in self.managed_resource_types:
            raise ValueError('Cannot scale resource type: %s' % resource_type)
        if desired_pods == current_pods:
            return None
        if resource_type == 'job':
            self.patch_namespaced_job(
                name, namespace, {'spec': {'parallelism': desired_pods}})
        else:
            self.patch_namespaced_deployment(
                name, namespace, {'spec': {'replicas': desired_pods}})
        self.logger.info('Successfully scaled %s `%s` in namespace `%s` '
                         'from %s to %s pods.', resource_type, name,
                         namespace, current_pods, desired_pods)
        self.events.emit('scale', kind=resource_type, name=name,
                         namespace=namespace, current=current_pods,
                         desired=desired_pods)
        return True

    # -- C14 -----------------------------------------------------------------
    def _decide(self, min_pods, max_pods, keys_per_pod, current_pods):
        if self.policy == 'reference':
            desired = 0
            for key in self.redis_keys:
                desired += self.get_desired_pods(key, keys_per_pod, min_pods,
                                                 max_pods, current_pods)
            return self.clip_pod_count(desired, min_pods, max_pods,
                                       current_pods)
        desired = policies.decide(
            self.redis_keys, min_pods, max_pods, keys_per_pod, current_pods,
            policy=self.policy, busy=len(self.busy_workers))
        delay = self.scale_down_delay
        if desired == 0:
            delay = max(delay, self.zero_delay)
        if desired < current_pods and delay > 0:
            now = self._clock()
            if self._lower_since is None:
                self._lower_since = now
            if now - self._lower_since < delay:
                # (a drop to zero still held: keep the workers but let a
                # lower non-zero target through at once)
                if desired == 0 and self.scale_down_delay <= 0:
                    return max(1, min(current_pods, desired or 1))
                return current_pods
        else:
            self._lower_since = None
        return desired

    def scale(self, namespace, resource_type, name, min_pods=0, max_pods=1,
              keys_per_pod=1):
        """One reconcile tick.  Returns the target replica count.

        Reference: ``autoscaler/autoscaler.py:244-273``."""
        tick_start = self._clock()
        self.tally_queues()
        self.logger.debug('Scaling %s `%s.%s`.', resource_type, namespace,
                          name)
        current_pods = self.get_current_pods(namespace, resource_type, name)
        desired_pods = self._decide(min_pods, max_pods, keys_per_pod,
                                    current_pods)
        self.logger.debug('%s `%s` in namespace `%s` has a current state of '
                          '%s pods and a desired state of %s pods.',
                          str(resource_type).capitalize(), name, namespace,
                          current_pods, desired_pods)
        tick_s = self._clock() - tick_start
        decided_ns = now_ns()
        self.last_decision = desired_pods
        try:
            self.scale_resource(desired_pods, current_pods, resource_type,
                                namespace, name)
        except ActuatorError as err:
            self.logger.warning('Failed to scale %s `%s.%s` due to %s: %s',
                                resource_type, namespace, name,
                                type(err).__name__, err)
        # stamped at the decision, sent after the actuator call: with a
        # Redis event sink the send is a round trip the PATCH need not wait
        # for (profiles/r5_boot)
        self.events.emit('tick', t_ns=decided_ns, keys=dict(self.redis_keys),
                         in_progress=dict(self.in_progress),
                         current=current_pods, desired=desired_pods,
                         tick_s=tick_s)
        return desired_pods
