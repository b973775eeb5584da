"""Manager side of the persistent node-wide membership communicator.

See :mod:`kiosk_autoscaler_amd.parallel.nodefence` for the protocol.  The
manager owns the communicator's *generation*: it starts one when every
managed GPU slot has a live process running a node agent (pool boot), relays
rank 0's communicator id to the other ranks, and breaks it -- ``comm_abort``
to the survivors, a fresh generation once the slot is repopulated -- only
when a slot's process dies or is retired.  Scale events never touch it: a
membership change is one ``fence`` all-reduce over the existing
communicator, serialized node-wide (every rank takes part in every
collective, in the same order).

This replaces the per-event ``ncclCommInitRank`` that the round-1 design
paid at every READY-set change (the actuation the fence gates is the
reference's ``patch_namespaced_*``, ``autoscaler/autoscaler.py:221-242``).
"""
import logging
import time

logger = logging.getLogger('NodeComm')

NONE, INIT, READY = 'none', 'init', 'ready'
# worker -> manager messages of the node agent (parallel.nodefence)
NODE_EVENTS = ('comm_uid', 'comm_ready', 'fenced', 'node_agent')


class NodeComm(object):
    def __init__(self, manager, init_timeout=120.0, fence_timeout=30.0,
                 fallback='store', fallback_after=2):
        self.m = manager
        # after ``fallback_after`` consecutive failed generations the next
        # ones use the ``fallback`` transport (every rank switches in its
        # ``comm_init``): membership stays fenced when RCCL cannot build the
        # node communicator; the JSON/metrics name the transport in use
        self.fallback = fallback or None
        self.fallback_after = max(1, int(fallback_after))
        self.transport_override = None
        self.init_timeout = float(init_timeout)
        self.fence_timeout = float(fence_timeout)
        self.gen = 0
        self.state = NONE
        self.members = []        # [(slot index, _Process)] in rank order
        self.ready_ranks = {}
        self.t_start = 0.0
        self.failures = 0
        self.retry_at = 0.0
        self.seq = 0             # node-wide fence sequence number
        self.inflight = None     # dict: resource, epoch, seq, members, t
        self.generations = 0     # communicators built (for tests/metrics)
        self.transport = None

    # ------------------------------------------------------------------
    @property
    def ready(self):
        return self.state == READY

    def _bound(self):
        """slot index -> the process currently serving that slot."""
        bound = {}
        for index, proc in self.m.standbys.items():
            bound[index] = proc
        for resource in self.m.resources.values():
            for worker in resource.workers.values():
                if worker.state != 'exited':
                    bound[worker.slot.index] = worker.proc
        return bound

    @staticmethod
    def _usable(proc):
        return (proc is not None and getattr(proc, 'node_ok', False) and
                not proc.eof and proc.popen.poll() is None)

    def candidates(self):
        """``[(slot, proc)]`` over every managed slot, or ``None`` while one
        of them has no live process with a node agent."""
        bound = self._bound()
        out = []
        for slot in self.m.slots:
            proc = bound.get(slot.index)
            if not self._usable(proc) or proc in self.m.retiring:
                return None
            out.append((slot.index, proc))
        return out

    # ------------------------------------------------------------------
    def step(self, now=None):
        """Called from every manager poll (under the manager lock)."""
        now = time.monotonic() if now is None else now
        if self.state in (INIT, READY):
            bound = self._bound()
            lost = [index for index, proc in self.members
                    if not self._usable(proc) or proc in self.m.retiring or
                    bound.get(index) is not proc]
            if lost:
                self.break_('slot(s) %s lost their process' % lost)
            elif self.state == INIT and now - self.t_start > self.init_timeout:
                self.break_('generation %d init timed out' % self.gen,
                            failed=True)
        if self.state == NONE and now >= self.retry_at:
            members = self.candidates()
            if members:
                self._start(members, now)
        if self.inflight is not None and \
                now - self.inflight['t'] > self.fence_timeout:
            seq = self.inflight['seq']
            for _, proc in self.members:
                proc.pipe.send({'cmd': 'fence_abort', 'seq': seq})
            self.break_('fence seq %d timed out' % seq, failed=True)

    def _start(self, members, now):
        self.gen += 1
        self.state = INIT
        self.members = list(members)
        self.ready_ranks = {}
        self.t_start = now
        n = len(members)
        for rank, (_, proc) in enumerate(members):
            message = {'cmd': 'comm_init', 'gen': self.gen, 'rank': rank,
                       'nranks': n}
            if self.transport_override:
                message['transport'] = self.transport_override
            proc.pipe.send(message)
        self.m.events.emit('node_comm_init', gen=self.gen, n=n,
                           slots=[index for index, _ in members],
                           pids=[proc.pid for _, proc in members],
                           transport=self.transport_override)
        logger.info('Node communicator generation %d: %d ranks.', self.gen, n)
        self.m._publish_pool()

    def break_(self, reason, failed=False):
        """Drop the current generation (survivors abort; a fence in flight
        is re-run on the next one)."""
        if self.state == NONE:
            return
        for _, proc in self.members:
            if not proc.eof and proc.popen.poll() is None:
                proc.pipe.send({'cmd': 'comm_abort', 'gen': self.gen})
        if self.inflight is not None:
            self.inflight['resource'].fence_wanted = True
            self.inflight = None
        self.state = NONE
        self.members = []
        now = time.monotonic()
        if failed:
            self.failures += 1
            self.retry_at = now + min(30.0, 0.25 * 2 ** min(self.failures - 1,
                                                             8))
            if (self.fallback and self.transport_override is None and
                    self.failures >= self.fallback_after):
                self.transport_override = self.fallback
                self.retry_at = now
                self.m.events.emit('node_comm_fallback', gen=self.gen,
                                   transport=self.fallback,
                                   failures=self.failures)
                logger.warning('Node communicator: %d failed generations, '
                               'falling back to the %s transport.',
                               self.failures, self.fallback)
        else:
            self.retry_at = now
        self.m.events.emit('node_comm_break', gen=self.gen, reason=reason,
                           failed=failed)
        logger.warning('Node communicator generation %d dropped: %s.',
                       self.gen, reason)
        self.m._publish_pool()

    # ------------------------------------------------------------------
    def on_message(self, proc, message):
        kind = message.get('ev')
        if kind == 'node_agent':
            proc.node_ok = True
            return
        gen = message.get('gen')
        if kind == 'comm_uid':
            if self.state == INIT and gen == self.gen:
                for _, other in self.members[1:]:
                    other.pipe.send({'cmd': 'comm_uid', 'gen': gen,
                                     'uid': message.get('uid')})
        elif kind == 'comm_ready':
            if self.state != INIT or gen != self.gen:
                return
            if not message.get('ok'):
                self.break_('rank %s failed to connect: %s' % (
                    message.get('rank'), message.get('detail')), failed=True)
                return
            self.ready_ranks[message.get('rank')] = message
            if len(self.ready_ranks) == len(self.members):
                self.state = READY
                self.failures = 0
                self.generations += 1
                self.transport = message.get('transport')
                init_ms = max(float(r.get('init_ms') or 0.0)
                              for r in self.ready_ranks.values())
                self.m.events.emit('node_comm_ready', gen=self.gen,
                                   n=len(self.members), init_ms=init_ms,
                                   transport=self.transport)
                logger.info('Node communicator generation %d ready (%d ranks,'
                            ' %.0f ms).', self.gen, len(self.members), init_ms)
                self.m._publish_pool()
        elif kind == 'fenced':
            inflight = self.inflight
            if inflight is None or message.get('seq') != inflight['seq']:
                return
            self.inflight = None
            resource = inflight['resource']
            if not message.get('ok'):
                logger.warning('Node fence seq %s failed: %s',
                               inflight['seq'], message.get('detail'))
                resource.fence_wanted = True
                self.break_('fence failed on rank %s' % message.get('rank'),
                            failed=True)
                return
            self.m._fence_completed(resource, inflight['epoch'],
                                    inflight['members'], inflight['t'],
                                    message)

    # ------------------------------------------------------------------
    def fence(self, resource, members):
        """Start one membership epoch of ``resource`` (caller checked
        ``ready`` and that nothing is in flight)."""
        self.seq += 1
        resource.epoch += 1
        slots = [resource.workers[wid].slot.index for wid in members]
        message = {'cmd': 'fence', 'epoch': resource.epoch, 'seq': self.seq,
                   'gen': self.gen, 'slots': slots,
                   'width': len(self.m.slots),
                   'group': '%s/%s' % (resource.namespace, resource.name)}
        for _, proc in self.members:
            proc.pipe.send(message)
        self.inflight = {'resource': resource, 'epoch': resource.epoch,
                         'seq': self.seq, 'members': list(members),
                         't': time.monotonic()}
        self.m.events.emit('fence_start', epoch=resource.epoch,
                           members=members, seq=self.seq, gen=self.gen)
