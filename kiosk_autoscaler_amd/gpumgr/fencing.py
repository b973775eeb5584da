"""Membership-fence orchestration of the node-local GPU manager (SURVEY
N4): which implementation fences a resource, starting epochs when its READY
set changes, their completion / failure / retry, quarantining a worker whose
rank stopped answering, and publishing the agreed set
(``kiosk:active:<ns>:<name>``).

A mixin of :class:`~.controller.GpuManager`; split out of
``controller.py``.  Every method runs under the manager
lock.
"""
import json
import logging
import time

from .nodecomm import NodeComm
from .process import DRAINING, EXITED

logger = logging.getLogger('GpuManager')

ACTIVE_KEY = 'kiosk:active:{ns}:{name}'
#: ``FENCE_COMM``: ``node`` -- one persistent communicator over every
#: slot's long-lived process, a membership change is one all-reduce
#: (needs a standby per slot and recycling); ``epoch`` -- each change
#: bootstraps a communicator over the READY workers (round-1 design)
FENCE_COMMS = ('node', 'epoch')


class FencingMixin(object):
    """Fence epochs per resource over the node communicator or per-epoch
    communicators (see the module doc)."""

    def _init_fencing(self, fence, fence_comm, fence_timeout,
                      fence_init_timeout, fence_fallback, fence_fallback_after,
                      fence_transport):
        self.fence_enabled = fence
        self.fence_timeout = fence_timeout
        if fence_comm not in FENCE_COMMS:
            raise ValueError('FENCE_COMM must be one of %s, got %r'
                             % (FENCE_COMMS, fence_comm))
        self.fence_comm = fence_comm
        self.node = None
        if not fence:
            return
        if fence_comm == 'node' and not self._node_comm_possible():
            # an explicit setting is honoured or refused loudly, never
            # swapped silently
            logger.warning(
                'FENCE_COMM=node needs a standby per GPU slot and worker '
                'recycling (WARM_POOL=%d for %d slots, recycle=%s): fencing '
                'each membership epoch with its own communicator instead.',
                self.pool_size, len(self.slots), self.recycle)
            self.fence_comm = 'epoch'
            self.events.emit('fence_comm', requested='node', used='epoch')
        if self.fence_comm != 'node':
            return
        # RCCL for every GPU pool, one that parks (deep idle) included: each
        # wake's generation is built after the woken worker is READY, its
        # engine was built before its agent joined, so RCCL's one-time load
        # on the agent's thread holds up no launch on the READY path
        # (profiles/r4_collision), and a generation of fresh processes gets
        # the first-generation budget.  ``fence_transport`` (FENCE) picks
        # another transport explicitly.
        transport = fence_transport
        self.node = NodeComm(self, fence_timeout=min(fence_timeout, 30.0),
                             init_timeout=fence_init_timeout,
                             fallback=fence_fallback,
                             fallback_after=fence_fallback_after,
                             transport=transport)

    def _node_comm_possible(self):
        return bool(self.recycle and self.pool_template is not None and
                    self.slots and self.pool_size >= len(self.slots))

    def quarantine_worker(self, resource, worker, reason):
        """A worker whose node agent stopped answering (``NodeComm``
        verdict): never killed while it may hold a key.  It leaves the
        fenced set at once (``available_replicas``, ``kiosk:active``), stops
        pulling (drained, not recycled: its process is not trusted as a
        standby again) and exits after its in-flight key; the reconcile
        starts a replacement.  Called under the manager lock."""
        worker.fenced_out = True
        worker.quarantined_at = time.monotonic()
        if worker.id in resource.fenced_members:
            resource.fenced_members = [m for m in resource.fenced_members
                                       if m != worker.id]
            self._publish_active(resource)
        resource.fence_wanted = True
        if worker.state == DRAINING:
            worker.proc.pipe.send({'cmd': 'drain', 'reason': reason,
                                   'recycle': False})
        else:
            self._drain(worker, reason, recycle=False)
        self.events.emit('worker_quarantined', worker=worker.id,
                         gpu=worker.slot.index, busy=worker.busy,
                         reason=reason)

    # ------------------------------------------------------------------
    # membership fence orchestration
    # ------------------------------------------------------------------
    def _maybe_fence(self, resource):
        if not self.fence_enabled:
            return
        if self.node is not None:
            self._maybe_node_fence(resource)
            return
        inflight = resource.fence_inflight
        if inflight is not None:
            epoch, members, started = inflight
            dead = [m for m in members if m not in resource.workers or
                    resource.workers[m].state == EXITED]
            if dead or time.monotonic() - started > self.fence_timeout:
                logger.warning('Fence epoch %d abandoned (%s).', epoch,
                               'member exited' if dead else 'timeout')
                for wid in members:
                    w = resource.workers.get(wid)
                    if w is not None and w.state != EXITED:
                        w.proc.pipe.send({'cmd': 'fence_abort',
                                          'epoch': epoch})
                resource.fence_inflight = None
                self._fence_failed(resource)
            else:
                return
        if not resource.fence_wanted or \
                time.monotonic() < resource.fence_retry_at:
            return
        members = sorted((w.id for w in resource.ready()),
                         key=lambda wid: resource.workers[wid].slot.index)
        resource.fence_wanted = False
        if members == resource.fenced_members:
            return
        if not members:
            resource.fenced_members = []
            resource.fenced_epoch = resource.epoch
            self._publish_active(resource)
            return
        resource.epoch += 1
        epoch = resource.epoch
        previous = list(resource.fenced_members)
        for rank, wid in enumerate(members):
            resource.workers[wid].proc.pipe.send({
                'cmd': 'fence', 'epoch': epoch, 'rank': rank,
                'members': members, 'previous': previous,
                'slots': [resource.workers[m].slot.index for m in members],
                'fresh': resource.fence_fresh,
                'group': '%s/%s' % (resource.namespace, resource.name)})
        resource.fence_inflight = (epoch, members, time.monotonic())
        self.events.emit('fence_start', epoch=epoch, members=members)

    def _node_fence_runnable(self):
        """A resource has a membership change the node communicator can
        fence right now (every member runs on one of its ranks)."""
        for resource in self.resources.values():
            if not resource.fence_wanted:
                continue
            members = [w for w in resource.ready()]
            if sorted(w.id for w in members) == sorted(
                    resource.fenced_members):
                continue
            if self.node.can_fence([w.proc for w in members]):
                return True
        return False

    def _maybe_node_fence(self, resource):
        """One 72-B all-reduce over the persistent communicator; waits
        (fence_wanted stays set) while a generation is being built or
        shrunk, another resource's epoch is in flight, or a member runs on a
        process that is not a rank yet (a replacement awaiting the regrow)."""
        if not resource.fence_wanted:
            return
        members = sorted((w.id for w in resource.ready()),
                         key=lambda wid: resource.workers[wid].slot.index)
        inflight = self.node.inflight
        if not members and (inflight is None or
                            inflight['resource'] is not resource):
            # nobody left to agree with: the empty set is published at
            # once, whether or not a communicator exists (a deep-idle pool
            # retires the last worker's process right after its drain)
            resource.fence_wanted = False
            if resource.fenced_members:
                resource.fenced_members = []
                resource.fenced_epoch = resource.epoch
                self._publish_active(resource)
            return
        if not self.node.ready or inflight is not None:
            return
        if not self.node.can_fence([resource.workers[wid].proc
                                    for wid in members]):
            return
        resource.fence_wanted = False
        if members == resource.fenced_members:
            return
        self.node.fence(resource, members)

    def _fence_failed(self, resource):
        """Retry with a fresh communicator after an exponential backoff, so
        a persistently failing bootstrap cannot spin on RCCL inits."""
        resource.fence_wanted = True
        resource.fence_fresh = True
        resource.fence_failures += 1
        delay = min(30.0, 0.25 * 2 ** min(resource.fence_failures - 1, 8))
        resource.fence_retry_at = time.monotonic() + delay
        self.events.emit('fence_retry', name=resource.name, delay_s=delay,
                         failures=resource.fence_failures)

    def _on_fenced(self, resource, message):
        inflight = resource.fence_inflight
        if inflight is None or message.get('epoch') != inflight[0]:
            return
        epoch, members, started = inflight
        resource.fence_inflight = None
        if not message.get('ok', False):
            logger.warning('Fence epoch %d failed: %s', epoch,
                           message.get('detail'))
            resource.fence_error = str(message.get('detail'))[:300]
            self._fence_failed(resource)
            return
        self._fence_completed(resource, epoch, members, started, message)

    def _fence_failed_node(self, resource, message):
        """A node fence failed (not a shrink's interrupt): visible in the
        resource's ``status.fence`` until an epoch succeeds."""
        resource.fence_failures += 1
        resource.fence_error = str(message.get('detail'))[:300]
        self.events.emit('fence_failed', name=resource.name,
                         detail=resource.fence_error,
                         failures=resource.fence_failures)

    def _fence_completed(self, resource, epoch, members, started, message):
        resource.fence_fresh = False
        resource.fence_failures = 0
        resource.fence_error = None
        resource.fenced_epoch = epoch
        resource.fenced_members = members
        self.events.emit('fence_done', epoch=epoch, members=members,
                         wall_s=time.monotonic() - started,
                         transport=message.get('transport'),
                         allreduce_us=message.get('allreduce_us'),
                         init_ms=message.get('init_ms'),
                         n=message.get('n'), mode=message.get('mode'),
                         gen=message.get('gen'))
        self._publish_active(resource)

    def _publish_active(self, resource):
        if self.redis is None:
            return
        try:
            self.redis.set(ACTIVE_KEY.format(ns=resource.namespace,
                                             name=resource.name),
                           json.dumps({'epoch': resource.fenced_epoch,
                                       'members': resource.fenced_members}))
        except Exception:  # pylint: disable=broad-except
            pass
