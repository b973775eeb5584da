"""Checkpoint / resume and Redis bookkeeping of the node-local GPU manager
(SURVEY §5.4): the persisted declared count per resource, adoption of it by
a restarted manager, requeue of a dead worker's (or an earlier manager's
orphaned) in-flight items, and the per-worker status hash.

A mixin of :class:`~.controller.GpuManager`; split out of
``controller.py``.
"""
import logging
import re
import time

from ..utils.keys import worker_of

logger = logging.getLogger('GpuManager')

WORKER_KEY = 'kiosk:worker:{id}'
STATE_KEY = 'kiosk:gpumgr:{ns}:{kind}:{name}'


class StateMixin(object):
    """Persisted state, orphan recovery, requeue (see the module doc)."""

    # ------------------------------------------------------------------
    # checkpoint / resume
    # ------------------------------------------------------------------
    def _state_key(self, resource):
        return STATE_KEY.format(ns=resource.namespace, kind=resource.kind,
                                name=resource.name)

    def _persist(self, resource):
        if self.redis is None:
            return
        try:
            key = self._state_key(resource)
            self.redis.hset(key, mapping={
                'declared': resource.declared,
                'generation': resource.generation,
                'epoch': resource.epoch,
                'succeeded': resource.succeeded,
                'failed': resource.failed,
                'updated_ns': time.monotonic_ns()})
            if self.state_ttl > 0:
                self.redis.expire(key, self.state_ttl)
        except Exception as err:  # pylint: disable=broad-except
            logger.warning('could not persist manager state: %s', err)

    def _restore(self, resource):
        if self.redis is None:
            return
        try:
            state = self.redis.hgetall(self._state_key(resource))
        except Exception as err:  # pylint: disable=broad-except
            logger.warning('could not read manager state: %s', err)
            return
        if not state:
            return
        resource.declared = int(state.get('declared', 0))
        resource.generation = int(state.get('generation', 0))
        resource.epoch = int(state.get('epoch', 0))
        resource.succeeded = int(state.get('succeeded', 0))
        resource.failed = int(state.get('failed', 0))
        self.events.emit('state_restored', name=resource.name,
                         declared=resource.declared)
        logger.info('Restored %s %s: declared=%d generation=%d.',
                    resource.kind, resource.name, resource.declared,
                    resource.generation)

    def recover_orphans(self, resource):
        """Requeue ``processing-<q>:<resource>-g*`` items whose worker is
        not one of ours (a previous manager instance died with them)."""
        if self.redis is None:
            return 0
        moved = 0
        # exact id shape <name>-g<slot>-<instance>-<seq>: a prefix match
        # would also take the live items of a resource named '<name>-g2'
        # sharing the queue (shared-daemon mode)
        ours = re.compile(r'^%s-g\d+-[0-9a-f]+-\d+$' % re.escape(resource.name))
        live = set(wid for r in self.resources.values() for wid in r.workers)
        for queue in resource.template.queues:
            pattern = 'processing-%s:%s-g*' % (queue, resource.name)
            try:
                for key in list(self.redis.scan_iter(match=pattern,
                                                     count=1000)):
                    wid = worker_of(key)
                    if wid in live or not ours.match(wid):
                        continue
                    while self.redis.rpoplpush(key, queue) is not None:
                        moved += 1
                    self.redis.delete(key)
            except Exception as err:  # pylint: disable=broad-except
                logger.error('orphan recovery failed: %s', err)
        if moved:
            self.events.emit('orphans_requeued', name=resource.name,
                             items=moved)
            logger.warning('Requeued %d orphaned in-flight items of %s.',
                           moved, resource.name)
        return moved

    def _requeue(self, resource, worker):
        """Push a dead worker's in-flight items back to their queues."""
        if self.redis is None:
            return 0
        moved = 0
        for queue in resource.template.queues:
            # exact key plus the per-slot keys of a batched pull; never a
            # bare prefix (worker 1 must not claim worker 12's items)
            exact = 'processing-%s:%s' % (queue, worker.id)
            try:
                keys = list(self.redis.scan_iter(match=exact + '.*',
                                                 count=1000))
                if self.redis.exists(exact):
                    keys.append(exact)
                for key in keys:
                    while self.redis.rpoplpush(key, queue) is not None:
                        moved += 1
                    self.redis.delete(key)
            except Exception as err:  # pylint: disable=broad-except
                logger.error('requeue of %s failed: %s', worker.id, err)
        if moved:
            self.events.emit('requeue', worker=worker.id, items=moved)
        return moved

    def _publish_worker(self, worker):
        if self.redis is None:
            return
        try:
            self.redis.hset(WORKER_KEY.format(id=worker.id), mapping={
                'gpu': worker.slot.index, 'pid': worker.proc.pid,
                'state': worker.state, 'ready_ns': worker.t_ready or 0,
                'resource': worker.resource.name})
        except Exception:  # pylint: disable=broad-except
            pass
