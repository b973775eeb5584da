"""Node-local GPU/process manager -- the Kubernetes replacement.

The reference's actuator is the Kubernetes API: it reads ``spec.replicas``
and PATCHes it, and k8s controllers create pods later
(``autoscaler/autoscaler.py:79-195, 221-242``).  On one 8-GPU MI355X node
this module plays API server + controller + kubelet:

* **Resources** (``deployment`` / ``job``) carry a declared count; a PATCH
  sets it and wakes the reconcile loop (no pod-scheduling round trip).
* **Workers** are OS processes, one per GPU, pinned with
  ``HIP_VISIBLE_DEVICES`` and CPU affinity to the GPU's NUMA-local cores.
  The lowest free GPU index is allocated first.
* **Warm pool**: ``pool_size`` standby processes, each pinned to its GPU
  at spawn, have imported the native kernel module (not PyTorch).  With
  ``WARM_POOL_MODE=device`` (the default) they have also created the HIP
  context and loaded every code object, so **a standby holds its GPU**
  (context and code objects, no weights; the benchmark reports this as
  ``standby_gpu_s``); with ``import`` they stop before HIP and hold none.
  A scale-up hands a standby its assignment over a pipe, taking process
  start, imports and the HIP init (0.27 s together) off the critical path
  (SURVEY §7.4 item 4).  Standbys do not count as replicas.
* **READY** (``status.available_replicas``) means the worker has its
  weights in HBM and has run the warm-start kernel.
* **Scale-down** drains: the worker finishes its in-flight key and exits.
  Busy workers are never chosen while an idle or not-ready one exists.
* **Failure**: a dead worker's ``processing-<q>:<id>*`` items are pushed
  back to their queue and a replacement is started (with backoff).
* **Jobs** are one-shot: workers exit 0 when the queue is empty; each
  success decrements ``spec.parallelism`` (TTL-after-finished semantics), so
  the reference's stranded-keys case (a completed Job that is never
  restarted) cannot occur.
* **Membership fence**: whenever the READY set changes the manager starts a
  fence epoch (coalesced: one in flight at a time); the set is agreed with
  a 72-B RCCL all-reduce over xGMI and rank 0 acknowledges.  With a standby
  per GPU the communicator is persistent (:mod:`.nodecomm`: built once over
  every slot's process, rebuilt only when one dies); otherwise each epoch
  bootstraps its own over the READY workers.  The fenced set is published
  to Redis (``kiosk:active:<ns>:<name>``).
"""
import collections
import itertools
import json
import logging
import os
import re
import select
import subprocess
import sys
import threading
import time

from ..utils.events import NULL as NULL_EVENTS
from ..utils.keys import worker_of
from .nodecomm import NODE_EVENTS, NodeComm
from .resources import ActuatorError, ResourceList, ResourceView, \
    desired_from_body

logger = logging.getLogger('GpuManager')

STARTING, READY, DRAINING, EXITED = 'starting', 'ready', 'draining', 'exited'
ACTIVE_KEY = 'kiosk:active:{ns}:{name}'
WORKER_KEY = 'kiosk:worker:{id}'
POOL_KEY = 'kiosk:pool'
SLOTS_KEY = 'kiosk:slots'
STATE_KEY = 'kiosk:gpumgr:{ns}:{kind}:{name}'


class WorkerTemplate(object):
    """What to run for a resource (the pod template analog)."""

    def __init__(self, queues=('predict',), module=None, env=None,
                 python=None, backend='auto', keys_per_pod=1):
        self.queues = list(queues)
        self.module = module or 'kiosk_autoscaler_amd.worker.main'
        self.env = dict(env or {})
        self.python = python or sys.executable
        self.backend = backend
        self.keys_per_pod = int(keys_per_pod)

    def to_dict(self):
        return {'queues': self.queues, 'module': self.module,
                'env': self.env, 'backend': self.backend,
                'keys_per_pod': self.keys_per_pod}


def _bare_worker(template):
    """Spawn with ``python -S``: our own HIP worker with the built-in engine,
    not importing torch (``WORKER_IMPORT_TORCH``), unless
    ``WORKER_PYTHON_SITE=1``."""
    def flag(name):
        value = template.env.get(name, os.environ.get(name, '0'))
        return str(value) not in ('0', '')
    return (template.backend == 'hip' and
            template.module == 'kiosk_autoscaler_amd.worker.main' and
            not flag('WORKER_ENGINE') and    # a plug-in may need packages
            not flag('WORKER_IMPORT_TORCH') and
            not flag('WORKER_PYTHON_SITE'))


class _Pipe(object):
    """Line-oriented JSON channel over a pair of pipe fds."""

    def __init__(self, cmd_w, ev_r):
        self.cmd_w = cmd_w
        self.ev_r = ev_r
        self._buf = b''
        os.set_blocking(ev_r, False)

    def send(self, message):
        data = (json.dumps(message) + '\n').encode()
        try:
            os.write(self.cmd_w, data)
            return True
        except OSError:
            return False

    def read_messages(self):
        out = []
        while True:
            try:
                chunk = os.read(self.ev_r, 65536)
            except BlockingIOError:
                break
            except OSError:
                chunk = b''
            if not chunk:
                out.append(None)  # EOF
                break
            self._buf += chunk
        while b'\n' in self._buf:
            line, self._buf = self._buf.split(b'\n', 1)
            if line.strip():
                try:
                    out.append(json.loads(line))
                except ValueError:
                    logger.warning('bad worker message %r', line[:200])
        return out

    def close(self):
        for fd in (self.cmd_w, self.ev_r):
            try:
                os.close(fd)
            except OSError:
                pass


# A pool that parks only after this long without demand wakes rarely: its
# node communicator stays on RCCL (one generation per wake, ~2 s of RCCL
# init that starts after the woken worker is READY); one that parks sooner
# fences over host shared memory (a generation per wake in ~0.3 ms).
RCCL_PARK_MIN_S = 60.0


class _Process(object):
    """A child process (standby or worker) and its control pipe."""

    _ids = itertools.count()

    def __init__(self, popen, pipe, role):
        self.popen = popen
        self.pipe = pipe
        self.role = role
        self.seq = next(self._ids)
        self.t_spawn = time.monotonic_ns()
        self.booted = False
        self.eof = False
        self.recycles = 0
        self.node_ok = False    # runs a node-communicator agent
        self.hbm_free = None    # free HBM bytes the standby measured
        self.woken = False      # spawned by an arrival wake (prebuilds)
        self.engine_cached = False  # standby holds a built engine

    @property
    def pid(self):
        return self.popen.pid


class Worker(object):
    __slots__ = ('id', 'resource', 'slot', 'proc', 'state', 'busy',
                 't_assigned', 't_ready', 't_exit', 'exit_code', 'from_pool',
                 'stages', 'last_beat', 'kill_reason', 'fenced_out')

    def __init__(self, wid, resource, slot, proc, from_pool):
        self.id = wid
        self.resource = resource
        self.slot = slot
        self.proc = proc
        self.state = STARTING
        self.busy = False
        self.t_assigned = time.monotonic_ns()
        self.t_ready = None
        self.t_exit = None
        self.exit_code = None
        self.from_pool = from_pool
        self.stages = {}
        self.last_beat = time.monotonic()   # last sign of progress
        self.kill_reason = None
        self.fenced_out = False     # an agreed membership excluded it

    def summary(self):
        return {'id': self.id, 'gpu': self.slot.index, 'pid': self.proc.pid,
                'state': self.state, 'busy': self.busy,
                'from_pool': self.from_pool, 't_assigned': self.t_assigned,
                't_ready': self.t_ready, 'stages': dict(self.stages),
                'exit_code': self.exit_code, 'killed': self.kill_reason,
                'fenced_out': self.fenced_out}


class Resource(object):
    def __init__(self, kind, namespace, name, template):
        self.kind = kind
        self.namespace = namespace
        self.name = name
        self.template = template
        self.declared = 0
        self.generation = 0
        self.workers = collections.OrderedDict()
        self.succeeded = 0
        self.failed = 0
        self.restart_backoff_until = 0.0
        self.consecutive_failures = 0
        # fence bookkeeping
        self.epoch = 0
        self.fenced_epoch = 0
        self.fenced_members = []
        self.fence_inflight = None   # (epoch, members, t_start)
        self.fence_wanted = False
        self.fence_fresh = False     # force re-init after a failed epoch
        self.fence_failures = 0      # consecutive failed/abandoned epochs
        self.fence_retry_at = 0.0    # monotonic s; backoff after failures
        self.fence_error = None      # detail of the last failed epoch
        self.fence_enabled = True

    @property
    def key(self):
        return (self.kind, self.namespace, self.name)

    def live(self):
        return [w for w in self.workers.values() if w.state in (STARTING,
                                                                READY)]

    def ready(self):
        return [w for w in self.workers.values() if w.state == READY]

    def fenced_ready(self):
        """READY workers that are in the last agreed (fenced) membership."""
        return [wid for wid in self.fenced_members
                if wid in self.workers and self.workers[wid].state == READY]

    def fence_status(self):
        ready = sorted(w.id for w in self.ready())
        return {'epoch': self.fenced_epoch,
                'in_sync': sorted(self.fenced_members) == ready,
                'pending': bool(self.fence_wanted or self.fence_inflight),
                'failures': self.fence_failures,
                'last_error': self.fence_error}

    def view(self):
        live = self.live()
        return ResourceView.build(
            self.kind, self.namespace, self.name, self.declared,
            ready=len([w for w in live if w.state == READY]),
            active=len(live), succeeded=self.succeeded, failed=self.failed,
            generation=self.generation, epoch=self.fenced_epoch,
            gpus=[w.slot.index for w in live],
            fenced=len(self.fenced_ready()) if self.fence_enabled else None,
            fence=self.fence_status() if self.fence_enabled else None)


class GpuManager(object):
    """In-process manager.  Thread-safe; ``start()`` runs its event loop.

    Args:
        slots: :class:`~.gpus.GpuSlot` list this manager may use.
        redis_client: used to requeue a dead worker's items and to publish
            worker/active-set state (optional for pure unit tests).
        pool_size: warm standby processes to keep (0 disables the pool).
        pool_template: template used to boot standbys (backend/module/env).
        events: :class:`~kiosk_autoscaler_amd.utils.EventLog`.
        fence: run membership fences on READY-set changes.
        fence_timeout: seconds before an unacknowledged fence is abandoned.
        worker_timeout: a *busy* worker that reports no progress (a served
            key) for this many seconds is presumed hung -- stuck kernel,
            deadlocked collective -- and is SIGKILLed; its in-flight items
            are requeued like any other death (0 = off).
        start_timeout: a worker that is not READY this long after its
            assignment is SIGKILLed (0 = off).
        recycle: a cleanly drained worker (or a finished job worker) frees
            its HBM and becomes its GPU's standby again, keeping the HIP
            context -- no process re-boot before the next scale-up there.
        pool_idle_release_s: deep idle -- with no demand for this long the
            standbys exit and the node holds no GPU (0 = never).
        pool_wake_poll_s: while the pool is parked (or idling toward it),
            read the managed queues' lengths this often; a new arrival
            refills the pool at once instead of at the scale-up tick.  The
            scaling decision is untouched (it stays with the INTERVAL tick):
            the standbys only get the rest of the tick phase -- INTERVAL / 2
            on average -- to open their devices, so the scale-up finds them
            booted (0 = off).
        pool_wake_lead_s: with the next tick's instant known
            (:meth:`note_next_tick`, the embedded autoscaler loop), a parked
            pool wakes this long before that tick rather than at the
            arrival: the standbys boot and prebuild in ~0.1-0.2 s (0.5 s for
            the PyTorch plug-in), so the GPU is held only for the lead, not
            for the rest of the tick phase (0 = wake at the arrival).
        pool_wake_hold_s: an arrival-woken pool is kept at least this long
            (the autoscaler's tick period and a margin: the tick that scales
            for the key must find it), whatever ``pool_idle_release_s``.
    """

    def __init__(self, slots, redis_client=None, pool_size=0,
                 pool_template=None, events=None, fence=True,
                 pool_mode='device', state_ttl=3600,
                 fence_timeout=60.0, max_restart_backoff=10.0,
                 worker_timeout=0.0, start_timeout=0.0, recycle=True,
                 fence_comm='node', pool_idle_release_s=0.0,
                 fence_fallback='shm', fence_fallback_after=2,
                 fence_init_timeout=12.0, fence_transport=None,
                 zygote=False, pool_wake_poll_s=0.0, pool_wake_hold_s=0.0,
                 pool_wake_lead_s=0.0):
        self.slots = list(slots)
        self.redis = redis_client
        self.pool_size = max(0, int(pool_size))
        self.pool_template = pool_template
        self.pool_mode = pool_mode
        self.state_ttl = int(state_ttl)
        self.events = events if events is not None else NULL_EVENTS
        self.fence_enabled = fence
        self.fence_timeout = fence_timeout
        self.max_restart_backoff = max_restart_backoff
        self.worker_timeout = float(worker_timeout or 0.0)
        self.start_timeout = float(start_timeout or 0.0)
        self.recycle = bool(recycle)
        self.retiring = []   # recycled processes told to exit
        # deep idle: after this long without demand the standbys exit and
        # the pool stays empty until the next scale-up (0 = never)
        self.pool_idle_release_s = float(pool_idle_release_s or 0.0)
        self.pool_parked = False
        self._last_demand = time.monotonic()
        self.pool_wake_poll_s = float(pool_wake_poll_s or 0.0)
        self.pool_wake_hold_s = float(pool_wake_hold_s or 0.0)
        self._wake_until = 0.0
        self.pool_wake_lead_s = float(pool_wake_lead_s or 0.0)
        self._next_tick = None    # monotonic instant of the next tick
        # spawn -> booted+prebuilt of recent arrival-woken standbys: the
        # lead adapts to it (1.5 x the slowest + 50 ms, capped by the knob)
        self._wake_boots = collections.deque(maxlen=8)
        self._wake_at = None      # a deferred arrival wake
        self._next_arrival_check = 0.0
        # queue -> length at the last check; reset to empty when demand
        # ends (a scale to zero implies empty queues, stranded keys aside),
        # so a key landing before the first check still counts as arrived
        self._queued = {}
        self.arrival_wakes = 0
        self.resources = collections.OrderedDict()
        self.standbys = collections.OrderedDict()   # slot index -> _Process
        self.lock = threading.RLock()
        self._thread = None
        self._stop = threading.Event()
        self._wake_r, self._wake_w = os.pipe()
        os.set_blocking(self._wake_r, False)
        self._worker_seq = itertools.count()
        # worker ids must not repeat across manager restarts (persisted
        # state, orphan recovery, events): <name>-g<slot>-<instance>-<seq>
        self.instance = '%x' % ((os.getpid() << 20 ^ time.time_ns() >> 10)
                                & 0xfffff)
        self._stopping = False
        # worker zygote (worker/zygote.py): spawns fork from a process that
        # imported the worker (and torch, for a plug-in) without the GPU
        self.zygote_enabled = bool(zygote)
        self.zygote = None
        self._zygote_restart_at = 0.0
        self.mapping_fixes = 0   # slots remapped after a PCI check
        self.history = []   # exited workers, for accounting
        # persistent node-wide communicator: needs one long-lived process
        # per slot (a standby for every GPU, recycled workers); otherwise
        # every epoch bootstraps its own communicator (round-1 mode).  In
        # every pool mode: standbys that hold no GPU (context / import) run
        # it over the native shared-memory transport instead of RCCL, which
        # would need a hardware queue and ~0.8 GiB of HBM per GPU
        # (profiles/r2_hbm_hold); so does a pool that parks (deep idle),
        # whose every wake is a new set of processes -- a new RCCL
        # communicator per wake cost 2.1 s on average (5.7 s max) at one
        # rank (profiles/r3_tiers/deep_idle_v2.json), the shared-memory one
        # a millisecond
        self.fence_comm = fence_comm
        self.node = None
        if (fence and fence_comm == 'node' and self.recycle and
                pool_template is not None and self.slots and
                self.pool_size >= len(self.slots)):
            transport = fence_transport
            if transport is None and pool_template.backend == 'hip' and \
                    (pool_mode != 'device' or
                     0 < self.pool_idle_release_s < RCCL_PARK_MIN_S):
                transport = 'shm'
            self.node = NodeComm(self, fence_timeout=min(fence_timeout, 30.0),
                                 init_timeout=fence_init_timeout,
                                 fallback=fence_fallback,
                                 fallback_after=fence_fallback_after,
                                 transport=transport)
        for resource in self.resources.values():
            resource.fence_enabled = bool(fence)

    # ------------------------------------------------------------------
    # API (the kubernetes AppsV1Api / BatchV1Api analogs)
    # ------------------------------------------------------------------
    def register(self, kind, namespace, name, template, restore=True):
        """Create (or update the template of) a managed resource.

        With ``restore`` the declared count persisted by a previous manager
        instance is re-adopted (the Deployment-survives-a-restart analog,
        SURVEY §5.4) and in-flight items of workers that no longer exist are
        pushed back to their queues."""
        if kind not in ('deployment', 'job'):
            raise ValueError('kind must be deployment or job, got %r' % kind)
        with self.lock:
            key = (kind, namespace, name)
            if key not in self.resources:
                resource = Resource(kind, namespace, name, template)
                resource.fence_enabled = bool(self.fence_enabled)
                self.resources[key] = resource
                if restore:
                    self._restore(resource)
                    self.recover_orphans(resource)
            else:
                self.resources[key].template = template
            return self.resources[key].view()

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

    def _list(self, kind, namespace):
        with self.lock:
            return ResourceList(items=[
                r.view() for r in self.resources.values()
                if r.kind == kind and r.namespace == namespace])

    def list_namespaced_deployment(self, namespace):
        return self._list('deployment', namespace)

    def list_namespaced_job(self, namespace):
        return self._list('job', namespace)

    def _patch(self, kind, name, namespace, body):
        declared = desired_from_body(kind, body)
        with self.lock:
            resource = self.resources.get((kind, namespace, name))
            if resource is None:
                raise ActuatorError(404, '%s "%s" not found in namespace "%s"'
                                    % (kind, name, namespace))
            if declared > len(self.slots):
                logger.warning('%s %s asks for %d workers but only %d GPU '
                               'slots exist; the rest stay pending', kind,
                               name, declared, len(self.slots))
            resource.declared = declared
            resource.generation += 1
            self._persist(resource)
            self.events.emit('patch', kind=kind, name=name, declared=declared)
            self._reconcile(resource)
            view = resource.view()
        self._wake()
        return view

    def patch_namespaced_deployment(self, name, namespace, body):
        return self._patch('deployment', name, namespace, body)

    def patch_namespaced_job(self, name, namespace, body):
        return self._patch('job', name, namespace, body)

    def status(self):
        with self.lock:
            return {
                'slots': [s.to_dict() for s in self.slots],
                'standbys': [{'pid': p.pid, 'booted': p.booted,
                              'slot': index}
                             for index, p in self.standbys.items()],
                'node_comm': (self.node.summary() if self.node is not None
                              else None),
                # deep idle: parked pool, arrival wakes, current wake lead
                'pool': {'parked': self.pool_parked,
                         'arrival_wakes': self.arrival_wakes,
                         'wake_lead_s': (self.wake_lead()
                                         if self.pool_idle_release_s > 0
                                         else None)},
                'resources': [dict(r.view().to_dict(), workers=[
                    w.summary() for w in r.workers.values()])
                    for r in self.resources.values()],
            }

    # ------------------------------------------------------------------
    # lifecycle
    # ------------------------------------------------------------------
    def start(self):
        if self._thread is None:
            if self.node is not None:
                # shared-memory segments of generations whose ranks all died
                # before joining (a crashed earlier manager's node)
                from ..parallel.nodefence import sweep_stale_shm
                stale = sweep_stale_shm(
                    older_than=max(300.0, 5 * self.node.init_timeout))
                if stale:
                    logger.warning('Removed %d stale node-communicator '
                                   'segment(s): %s', len(stale), stale)
            with self.lock:
                self._start_zygote()
                self._refill_pool()
            self._thread = threading.Thread(target=self._loop,
                                            name='gpumgr', daemon=True)
            self._thread.start()
        return self

    def _wake(self):
        try:
            os.write(self._wake_w, b'x')
        except OSError:
            pass

    def _loop(self):
        while not self._stop.is_set():
            timeout = 0.05
            wake_at = self._wake_at
            if wake_at is not None:
                # a deferred arrival wake is due: do not sleep past it
                timeout = min(timeout, max(0.001, wake_at - time.monotonic()))
            self.poll(timeout)

    def stop(self, timeout=10.0):
        """Drain every worker, stop standbys, join the loop."""
        with self.lock:
            self._stopping = True
            for resource in self.resources.values():
                resource.declared = 0
                self._reconcile(resource)
            for proc in self.standbys.values():
                proc.pipe.send({'cmd': 'exit'})
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            with self.lock:
                alive = [w for r in self.resources.values()
                         for w in r.workers.values() if w.state != EXITED]
                alive += [p for p in self.standbys.values()
                          if p.popen.poll() is None]
                alive += [p for p in self.retiring
                          if p.popen.poll() is None]
            if not alive:
                break
            if self._thread is None:
                self.poll(0.05)
            else:
                time.sleep(0.05)
        with self.lock:
            for resource in self.resources.values():
                for worker in resource.workers.values():
                    if worker.proc.popen.poll() is None:
                        worker.proc.popen.kill()
            for proc in list(self.standbys.values()) + self.retiring:
                if proc.popen.poll() is None:
                    proc.popen.kill()
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
            self._thread = None
        with self.lock:
            self._reap_all()
            if self.zygote is not None:
                self.zygote.close()
                self.zygote = None

    # ------------------------------------------------------------------
    # event loop body
    # ------------------------------------------------------------------
    def poll(self, timeout=0.05):
        with self.lock:
            fds = {self._wake_r: None}
            for proc in self.standbys.values():
                if not proc.eof:
                    fds[proc.pipe.ev_r] = proc
            for resource in self.resources.values():
                for worker in resource.workers.values():
                    if worker.state != EXITED and not worker.proc.eof:
                        fds[worker.proc.pipe.ev_r] = worker
        try:
            ready, _, _ = select.select(list(fds), [], [], timeout)
        except (OSError, ValueError):
            ready = []
        with self.lock:
            for fd in ready:
                owner = fds.get(fd)
                if owner is None:
                    try:
                        os.read(self._wake_r, 4096)
                    except OSError:
                        pass
                elif isinstance(owner, _Process):
                    self._on_standby_messages(owner)
                else:
                    self._on_worker_messages(owner)
            self._reap_all()
            self._watchdog()
            if self.zygote_enabled and not self._check_zygote():
                self._start_zygote()      # a dead zygote, after a pause
            if self.node is not None and not self._stopping:
                self.node.step()
            for resource in self.resources.values():
                self._reconcile(resource)
                self._maybe_fence(resource)
            self._refill_pool()

    # ------------------------------------------------------------------
    # process management
    # ------------------------------------------------------------------
    @staticmethod
    def _interpreter(template):
        argv = [template.python]
        if _bare_worker(template):
            # the torch-free HIP worker needs only this tree (on PYTHONPATH
            # below) and the stdlib: skipping site-packages' .pth
            # processing takes ~20 ms off every spawn
            argv.append('-S')
        return argv

    @staticmethod
    def _environment(template):
        env = dict(os.environ)
        env.update({k: str(v) for k, v in template.env.items()})
        env['PYTHONUNBUFFERED'] = '1'
        root = os.path.dirname(os.path.dirname(os.path.dirname(
            os.path.abspath(__file__))))
        env['PYTHONPATH'] = os.pathsep.join(
            [root] + [p for p in env.get('PYTHONPATH', '').split(os.pathsep)
                      if p])
        return env

    # env that decides what a worker imports: a zygote serves only the
    # templates it preloaded for
    _IMPORT_ENV = ('WORKER_ENGINE', 'WORKER_IMPORT_TORCH', 'KIOSK_NATIVE',
                   'WORKER_PYTHON_SITE')

    def _start_zygote(self):
        tpl = self.pool_template
        if not self.zygote_enabled or tpl is None or self.zygote is not None \
                or tpl.module != 'kiosk_autoscaler_amd.worker.main' or \
                self._stopping or time.monotonic() < self._zygote_restart_at:
            return
        from ..worker import zygote
        if not zygote.become_subreaper():
            logger.warning('PR_SET_CHILD_SUBREAPER refused: no zygote.')
            self.zygote_enabled = False
            return
        argv = self._interpreter(tpl) + [
            '-m', 'kiosk_autoscaler_amd.worker.zygote', '--backend',
            tpl.backend]
        self.zygote = zygote.ZygoteClient(argv, self._environment(tpl))
        self.events.emit('zygote_spawn', pid=self.zygote.pid)

    def _check_zygote(self):
        """False (and the zygote forgotten, restarted after a pause) once
        the zygote process has exited."""
        z = self.zygote
        if z is None:
            return False
        if z.alive():
            return True
        logger.warning('Worker zygote %d exited; spawning directly until it '
                       'is restarted.', z.pid)
        self.events.emit('zygote_exit', pid=z.pid, code=z.popen.returncode)
        z.close()
        self.zygote = None
        self._zygote_restart_at = time.monotonic() + 10.0
        return False

    def _zygote_for(self, template):
        z = self.zygote
        tpl = self.pool_template
        if z is None or tpl is None:
            return None
        if not self._check_zygote():
            return None
        if not z.poll_ready():
            return None      # still importing: this spawn takes the slow path
        if (template.module != tpl.module or
                template.backend != tpl.backend or
                _bare_worker(template) != _bare_worker(tpl) or
                any(template.env.get(k) != tpl.env.get(k)
                    for k in self._IMPORT_ENV)):
            return None
        return z

    def _spawn(self, template, role, assign=None, slot=None):
        cmd_r, cmd_w = os.pipe()
        ev_r, ev_w = os.pipe()
        args = ['--cmd-fd', str(cmd_r), '--ev-fd', str(ev_w),
                '--backend', template.backend]
        # a standby spawned by an arrival wake: the scale-up for the key is
        # due within a tick, so it builds the engine now, not at the assign
        woken = (assign is None and slot is not None and role == 'standby'
                 and time.monotonic() < self._wake_until)
        if assign is not None:
            args += ['--assign', json.dumps(assign)]
        elif slot is not None:
            pin = {'gpu': slot.visible_id, 'slot': slot.index,
                   'cpus': slot.cpus, 'preinit': self.pool_mode,
                   'node_fence': self.node is not None}
            if woken:
                pin['prebuild'] = self._prebuild_spec(template)
            args += ['--pin', json.dumps(pin)]
        env = self._environment(template)
        popen = None
        via = 'exec'
        try:
            zygote = self._zygote_for(template)
            if zygote is not None:
                try:
                    popen = zygote.fork(args, env, (cmd_r, ev_w))
                    via = 'zygote'
                except (OSError, ValueError) as err:
                    logger.warning('zygote fork failed (%s); spawning '
                                   'directly.', err)
            if popen is None:
                argv = self._interpreter(template) + ['-m', template.module]
                popen = subprocess.Popen(argv + args, env=env,
                                         pass_fds=(cmd_r, ev_w),
                                         close_fds=True,
                                         start_new_session=True)
        finally:
            os.close(cmd_r)
            os.close(ev_w)
        proc = _Process(popen, _Pipe(cmd_w, ev_r), role)
        proc.woken = woken
        proc.slot = slot.index if slot is not None else None
        proc.via = via
        self.events.emit('process_spawn', role=role, pid=popen.pid,
                         slot=proc.slot, via=via)
        return proc

    def _refill_pool(self):
        """Keep one standby pinned to each of the lowest ``pool_size`` free
        GPUs (the slots the next scale-up will take)."""
        if not self.pool_size or self.pool_template is None or \
                self._stopping:
            return
        changed = False
        if self._reap_standbys():
            changed = True
        if self._park_pool():
            changed = True
        if self.pool_parked:
            if changed:
                self._publish_pool()
            return
        for slot in self._free_slots()[:self.pool_size]:
            if slot.index not in self.standbys:
                self.standbys[slot.index] = self._spawn(
                    self.pool_template, 'standby', slot=slot)
                changed = True
        if changed:
            self._publish_pool()

    def _park_pool(self):
        """Deep idle (``POOL_IDLE_RELEASE_S``): with no declared or live
        worker for that long, retire every standby -- the node then holds
        no GPU, like the reference at zero replicas -- and keep the pool
        empty until demand returns: a key's arrival (``pool_wake_poll_s``,
        woken ``wake_lead()`` before the next tick) or, without it, the
        scale-up itself, which is then a cold spawn with the pool refilling
        behind it.  True if standbys were retired."""
        now = time.monotonic()
        demand = any(r.declared > 0 or any(w.state != EXITED
                                           for w in r.workers.values())
                     for r in self.resources.values())
        if demand:
            self._last_demand = now
            self._queued = {}
            self._wake_at = None
            self._wake_until = 0.0    # the tick scaled: the hold is done
            if self.pool_parked:
                self.pool_parked = False
                self.events.emit('pool_resumed')
                logger.info('Demand returned: refilling the warm pool.')
            return False
        released = [p for p in self.standbys.values()
                    if p.booted and not p.engine_cached and
                    self.pool_mode == 'device']
        arrived = (self.pool_idle_release_s > 0 or bool(released)) and \
            self._arrived(now)
        if arrived and released:
            # ENGINE_IDLE_RELEASE_S freed these standbys' engines: a key's
            # arrival has them rebuild it before the scale-up tick
            for proc in released:
                proc.pipe.send({'cmd': 'prebuild',
                                'spec': self._prebuild_spec(
                                    self.pool_template)})
                proc.engine_cached = True     # (until told otherwise)
            self.events.emit('engine_rebuild', standbys=len(released))
        if arrived and self.pool_idle_release_s > 0:
            wake_at = now
            lead = self.wake_lead()
            if self.pool_parked and lead > 0 and \
                    self._next_tick is not None and \
                    self._next_tick - now > lead:
                wake_at = self._next_tick - lead
            if self._wake_at is None or wake_at < self._wake_at:
                self._wake_at = wake_at
        if self._wake_at is not None and now >= self._wake_at:
            self._wake_at = None
            self._last_demand = now
            self._wake_until = now + self.pool_wake_hold_s
            if self.pool_parked:
                self.pool_parked = False
                self.arrival_wakes += 1
                self.events.emit('pool_resumed', reason='arrival',
                                 lead_s=round(self.wake_lead(), 4),
                                 tick_in_s=(round(self._next_tick - now, 4)
                                            if self._next_tick is not None
                                            else None))
                logger.info('Keys arrived: refilling the warm pool ahead of '
                            'the scale-up tick.')
            return False
        if (self.pool_idle_release_s <= 0 or self.pool_parked or
                now - self._last_demand < self.pool_idle_release_s or
                now < self._wake_until):
            return False
        self.pool_parked = True
        released = 0
        for index, proc in list(self.standbys.items()):
            if proc.popen.poll() is None:
                proc.pipe.send({'cmd': 'exit'})
                self.retiring.append(proc)
                released += 1
            del self.standbys[index]
        self.events.emit('pool_parked', standbys=released,
                         idle_s=round(now - self._last_demand, 3))
        logger.info('No demand for %.0f s: released %d standby process(es).',
                    now - self._last_demand, released)
        return True

    def note_next_tick(self, t_monotonic):
        """The autoscaler loop's next tick instant (``time.monotonic``
        seconds, system-wide, so a ``unix:`` daemon's clients report it
        too): a deferred arrival wake is timed against it.  With several
        autoscalers on one manager the earliest upcoming tick wins (a
        report replaces a tick that is due or past).  Called from the
        loop's thread: under the manager lock."""
        t_monotonic = float(t_monotonic)
        with self.lock:
            current = self._next_tick
            if current is None or current <= time.monotonic() + 0.05 or \
                    t_monotonic < current:
                self._next_tick = t_monotonic
            lead = self.wake_lead()
            if self._wake_at is not None and lead > 0:
                # the tick came earlier than planned for (IDLE_INTERVAL)
                self._wake_at = min(self._wake_at, self._next_tick - lead)
        self._wake()

    def wake_lead(self):
        """Seconds before the next tick an arrival wakes a parked pool:
        ``pool_wake_lead_s`` until woken standbys have been timed, then
        1.5 x the slowest of the last 8 spawn -> booted+prebuilt times plus
        50 ms and the arrival poll, at least 0.2 s, never above
        ``pool_wake_lead_s`` (built-in worker: ~0.1-0.2 s -> 0.25-0.4 s;
        PyTorch plug-in: ~0.55 s -> the cap)."""
        cap = self.pool_wake_lead_s
        if cap <= 0 or not self._wake_boots:
            return cap
        return min(cap, max(0.2, 1.5 * max(self._wake_boots) + 0.05 +
                            self.pool_wake_poll_s))

    def _prebuild_spec(self, template):
        """What an arrival-woken standby builds its engine for: the shape
        (kind, keys per pod) of the resource its template serves."""
        for resource in self.resources.values():
            if resource.template.module == template.module:
                return {'kind': resource.kind,
                        'keys_per_pod': resource.template.keys_per_pod}
        return {'kind': 'deployment', 'keys_per_pod': template.keys_per_pod}

    def _arrived(self, now):
        """True when a managed queue grew since the last check (read every
        ``pool_wake_poll_s`` while no worker is declared or live).  Growth,
        not length: keys a policy strands below KEYS_PER_POD do not hold
        the pool, new ones wake it.  One pipelined LLEN per queue."""
        if self.pool_wake_poll_s <= 0 or self.redis is None or \
                now < self._next_arrival_check:
            return False
        self._next_arrival_check = now + self.pool_wake_poll_s
        queues = sorted(set(q for r in self.resources.values()
                            for q in r.template.queues))
        if not queues:
            return False
        try:
            pipe = self.redis.pipeline(transaction=False)
            for queue in queues:
                pipe.llen(queue)
            lengths = dict(zip(queues, (int(n or 0) for n in pipe.execute())))
        except Exception as err:  # pylint: disable=broad-except
            logger.debug('arrival check failed: %s', err)
            return False
        before, self._queued = self._queued, lengths
        grown = [q for q in queues if lengths[q] > before.get(q, 0)]
        if grown:
            self.events.emit('arrival', queues=grown,
                             parked=self.pool_parked)
        return bool(grown)

    def _take_standby(self, template, slot):
        """The standby pinned to ``slot`` (booted or still booting: it
        reads the assignment as soon as its imports finish)."""
        if self.pool_template is None or \
                template.module != self.pool_template.module or \
                template.backend != self.pool_template.backend:
            return None
        proc = self.standbys.get(slot.index)
        if proc is None or proc.popen.poll() is not None:
            return None
        del self.standbys[slot.index]
        self._publish_pool()
        return proc

    def _publish_slots(self):
        """The slot table as verified so far (``kiosk:slots``): the bench
        samples amdsmi on these PCI addresses, not on KFD order."""
        if self.redis is None:
            return
        try:
            self.redis.set(SLOTS_KEY, json.dumps([
                {'index': s.index, 'visible': s.visible_id, 'pci': s.pci,
                 'verified': bool(getattr(s, 'pci_verified', False)),
                 'kind': s.kind} for s in self.slots]))
        except Exception:  # pylint: disable=broad-except
            pass

    def _publish_pool(self):
        if self.redis is None:
            return
        try:
            # booted standbys, standbys, node communicator state, parked
            # (POOL_IDLE_RELEASE_S: the pool is empty on purpose)
            self.redis.set(POOL_KEY, '%d %d %s %d' % (
                sum(1 for p in self.standbys.values() if p.booted),
                len(self.standbys),
                self.node.state if self.node is not None else 'off',
                int(self.pool_parked)))
        except Exception:  # pylint: disable=broad-except
            pass

    def _on_standby_messages(self, proc):
        for message in proc.pipe.read_messages():
            if message is None:
                proc.eof = True
                continue
            self._on_standby_message(proc, message)

    def _on_standby_message(self, proc, message):
        if self.node is not None and message.get('ev') in NODE_EVENTS:
            self.node.on_message(proc, message)
            return
        if message.get('ev') == 'engine_released':
            proc.engine_cached = False
            proc.hbm_free = message.get('hbm_free')
            self.events.emit('engine_released', pid=proc.pid, slot=proc.slot,
                             released_bytes=message.get('released_bytes'),
                             hbm_free=proc.hbm_free)
            return
        if message.get('ev') == 'device':
            self._check_device(proc, message.get('pci'))
            return
        if message.get('ev') == 'prebuilt':
            proc.engine_cached = not message.get('error')
            self.events.emit('standby_prebuilt', pid=proc.pid, slot=proc.slot,
                             ms=message.get('ms'),
                             hbm_bytes=message.get('hbm_bytes'),
                             error=message.get('error'))
            return
        if message.get('ev') == 'standby':
            proc.engine_cached = bool(message.get('engine_cached'))
            if proc.woken and not proc.booted:
                # spawn -> booted and prebuilt: what the wake lead must cover
                # (once: a recycled worker reports 'standby' again later)
                proc.woken = False
                self._wake_boots.append(
                    (time.monotonic_ns() - proc.t_spawn) / 1e9)
            proc.booted = True
            proc.hbm_free = message.get('hbm_free')
            if message.get('pci'):
                if not self._check_device(proc, message.get('pci')):
                    return   # retired: the pool respawns it re-pinned
            self._publish_pool()
            self.events.emit('standby_ready', pid=proc.pid, slot=proc.slot,
                             boot_s=(time.monotonic_ns() - proc.t_spawn)
                             / 1e9, preinit=message.get('preinit'),
                             recycled=proc.role == 'standby' and
                             proc.recycles > 0)

    def _check_device(self, proc, pci):
        """the slot table maps slot -> HIP ordinal -> PCI address
        from KFD topology order, which drives the HIP_VISIBLE_DEVICES pin,
        the NUMA-local CPU affinity and the BDF the benchmark's amdsmi
        cross-check samples.  The process reports the PCI address HIP sees
        for its ordinal; on a mismatch the slot is remapped to the device
        actually behind that ordinal (its NUMA node and CPUs re-read) and a
        standby pinned with the wrong affinity is respawned.  False when
        ``proc`` was retired for that."""
        from .gpus import local_cpus, normalize_pci
        index = proc.slot
        slot = next((s for s in self.slots if s.index == index), None)
        actual = normalize_pci(pci)
        if slot is None or slot.kind != 'gpu' or actual is None:
            return True
        expected = normalize_pci(slot.pci)
        proc.pci = actual
        if expected == actual:
            if not getattr(slot, 'pci_verified', False):
                slot.pci_verified = True
                self.events.emit('gpu_mapping', slot=index, pci=actual,
                                 visible=slot.visible_id, verified=True)
                self._publish_slots()
            return True
        slot.pci = actual
        slot.numa_node, slot.cpus = local_cpus(actual)
        slot.pci_verified = True
        self.mapping_fixes += 1
        self.events.emit('gpu_mapping_mismatch', slot=index,
                         visible=slot.visible_id, expected=expected,
                         actual=actual, numa_node=slot.numa_node)
        logger.error('GPU slot %d (HIP_VISIBLE_DEVICES=%s) is %s, not %s as '
                     'KFD order suggested: remapped (NUMA node %s).', index,
                     slot.visible_id, actual, expected, slot.numa_node)
        self._publish_slots()
        if self.standbys.get(index) is proc and expected is not None:
            del self.standbys[index]
            proc.pipe.send({'cmd': 'exit'})
            self.retiring.append(proc)
            return False
        return True

    def _recycle_ok(self, resource):
        tpl = self.pool_template
        return bool(self.recycle and self.pool_size and tpl is not None and
                    not self._stopping and
                    resource.template.module == tpl.module and
                    resource.template.backend == tpl.backend)

    def _on_recycled(self, worker, message):
        """A worker finished cleanly and kept its process: account for it
        like an exit, then adopt the process as its GPU's standby."""
        if worker.state == EXITED:
            return
        resource = worker.resource
        proc = worker.proc
        self._on_exit(resource, worker, int(message.get('code', 0)),
                      recycled=True)
        slot = worker.slot
        proc.recycles += 1
        if (self._recycle_ok(resource) and slot.index not in self.standbys
                and len(self.standbys) < self.pool_size):
            proc.role = 'standby'
            proc.slot = slot.index
            proc.booted = False     # until its 'standby' message
            self.standbys[slot.index] = proc
            self._publish_pool()
            self.events.emit('worker_recycled', worker=worker.id,
                             gpu=slot.index, pid=proc.pid)
        else:
            proc.pipe.send({'cmd': 'exit'})
            self.retiring.append(proc)

    def _free_slots(self):
        used = set()
        for resource in self.resources.values():
            for worker in resource.workers.values():
                if worker.state != EXITED:
                    used.add(worker.slot.index)
        return [s for s in self.slots if s.index not in used]

    def _start_worker(self, resource, slot):
        wid = '%s-g%d-%s-%d' % (resource.name, slot.index, self.instance,
                                next(self._worker_seq))
        assign = {
            'cmd': 'assign', 'worker_id': wid, 'gpu': slot.visible_id,
            'slot': slot.index, 'cpus': slot.cpus, 'kind': resource.kind,
            'namespace': resource.namespace, 'resource': resource.name,
            'template': resource.template.to_dict(),
            't_assign': time.monotonic_ns(),
            'recycle': self._recycle_ok(resource),
            'node_fence': self.node is not None,
        }
        proc = self._take_standby(resource.template, slot)
        from_pool = proc is not None
        if from_pool and proc.hbm_free:
            self._size_from_free(resource, assign, proc.hbm_free, slot)
        if from_pool:
            if not proc.pipe.send(assign):
                proc.popen.kill()
                proc = None
                from_pool = False
        if proc is None:
            proc = self._spawn(resource.template, 'worker', assign=assign,
                               slot=slot)
        proc.role = 'worker'
        worker = Worker(wid, resource, slot, proc, from_pool)
        resource.workers[wid] = worker
        self.events.emit('worker_assigned', worker=wid, gpu=slot.index,
                         pid=proc.pid, from_pool=from_pool,
                         resource=resource.name)
        logger.info('Started worker %s on GPU %s (pid %d, %s).', wid,
                    slot.visible_id or slot.index, proc.pid,
                    'warm pool' if from_pool else 'cold spawn')
        return worker

    def _size_from_free(self, resource, assign, free, slot):
        """N5: clamp this assignment's KEYS_PER_POD (the job worker's batch)
        to what fits in the HBM the standby measured free."""
        from ..utils import hbm
        tpl = resource.template
        env = tpl.env

        def num(name, default):
            try:
                return int(env.get(name, default))
            except (TypeError, ValueError):
                return default
        kpp, limit = hbm.size_from_free(
            tpl.keys_per_pod, free, num('MODEL_DIM', 4096),
            num('MODEL_HIDDEN', 16384), num('MODEL_LAYERS', 4),
            num('ROWS_PER_KEY', 2048),
            reserve=num('HBM_FREE_RESERVE_BYTES', 1 << 30),
            per_key=num('HBM_PER_KEY_BYTES', 0))
        if kpp != tpl.keys_per_pod:
            logger.warning('KEYS_PER_POD=%d does not fit the %.1f GB free on '
                           'GPU %s (max %d); this worker batches %d',
                           tpl.keys_per_pod, free / 1e9, slot.index, limit,
                           kpp)
        assign['template'] = dict(assign['template'], keys_per_pod=kpp)
        self.events.emit('hbm_sizing', gpu=slot.index, hbm_free=free,
                         max_keys_per_pod=limit, keys_per_pod=kpp,
                         requested=tpl.keys_per_pod)

    def _drain(self, worker, reason):
        if worker.state in (DRAINING, EXITED):
            return
        worker.state = DRAINING
        worker.proc.pipe.send({'cmd': 'drain', 'reason': reason,
                               'recycle': self._recycle_ok(worker.resource)})
        self.events.emit('worker_drain', worker=worker.id, reason=reason)
        logger.info('Draining worker %s (%s).', worker.id, reason)

    def _reconcile(self, resource):
        live = resource.live()
        if len(live) < resource.declared and not self._stopping:
            # a deployment scaling back up while one of its workers is still
            # draining: cancel the drain instead of waiting for the process
            # to leave and starting over (if the worker has already left its
            # serving loop, it reports `recycled` and is replaced as usual)
            if resource.kind == 'deployment':
                for worker in resource.workers.values():
                    if len(live) >= resource.declared:
                        break
                    if worker.state == DRAINING and not worker.kill_reason \
                            and worker.t_ready:
                        if worker.proc.pipe.send({'cmd': 'undrain'}):
                            worker.state = READY
                            live.append(worker)
                            self.events.emit('worker_undrain',
                                             worker=worker.id)
                            logger.info('Cancelled the drain of worker %s.',
                                        worker.id)
                if len(live) >= resource.declared:
                    return
            if time.monotonic() < resource.restart_backoff_until:
                return
            free = self._free_slots()
            for slot in free[:resource.declared - len(live)]:
                self._start_worker(resource, slot)
        elif len(live) > resource.declared:
            excess = len(live) - resource.declared
            # victims: not-ready first, then idle; newest first; busy last
            order = sorted(live, key=lambda w: (
                w.state == READY, w.busy, -w.t_assigned))
            for worker in order:
                if excess == 0:
                    break
                if worker.busy and any(not w.busy for w in order
                                       if w.state != DRAINING):
                    continue
                self._drain(worker, 'scale-down')
                excess -= 1

    def _on_worker_messages(self, worker):
        for message in worker.proc.pipe.read_messages():
            if message is None:
                worker.proc.eof = True
                continue
            kind = message.get('ev')
            if self.node is not None and kind in NODE_EVENTS:
                self.node.on_message(worker.proc, message)
            elif kind == 'stage':
                worker.stages[message.get('stage')] = message.get('t')
            elif kind == 'ready':
                if worker.state == STARTING:
                    worker.state = READY
                worker.t_ready = message.get('t', time.monotonic_ns())
                worker.stages.update(message.get('stages', {}))
                worker.resource.fence_wanted = True
                worker.resource.consecutive_failures = 0
                self._publish_worker(worker)
                self.events.emit('worker_up', worker=worker.id,
                                 gpu=worker.slot.index,
                                 from_pool=worker.from_pool,
                                 resource=worker.resource.name,
                                 ready_s=(worker.t_ready -
                                          worker.t_assigned) / 1e9)
                logger.info('Worker %s READY on GPU %s after %.3f s.',
                            worker.id, worker.slot.index,
                            (worker.t_ready - worker.t_assigned) / 1e9)
            elif kind == 'busy':
                worker.busy = True
                worker.last_beat = time.monotonic()
            elif kind == 'beat':
                worker.last_beat = time.monotonic()
            elif kind == 'idle':
                worker.busy = False
                worker.last_beat = time.monotonic()
            elif kind == 'fenced':
                self._on_fenced(worker.resource, message)
            elif kind in ('fenced_out', 'fenced_in'):
                worker.fenced_out = kind == 'fenced_out'
                self.events.emit('worker_' + kind, worker=worker.id,
                                 seq=message.get('seq'))
            elif kind == 'recycled':
                self._on_recycled(worker, message)
            elif kind in ('standby', 'device'):
                # the rest of a batch that also held 'recycled'; a cold
                # spawn's device report
                self._on_standby_message(worker.proc, message)
            elif kind == 'error':
                logger.error('Worker %s reported: %s', worker.id,
                             message.get('message'))

    def _watchdog(self):
        """Failure detection beyond waitpid: kill workers that
        are alive but stuck.  The kill is an ordinary death afterwards --
        reaped, items requeued, restart backoff, fence re-run."""
        if not (self.worker_timeout or self.start_timeout):
            return
        now = time.monotonic()
        for resource in self.resources.values():
            for worker in resource.workers.values():
                if worker.state == EXITED or worker.kill_reason:
                    continue
                reason = None
                if (self.start_timeout and worker.state == STARTING and
                        now - worker.t_assigned / 1e9 > self.start_timeout):
                    reason = 'not READY after %.1f s' % self.start_timeout
                elif (self.worker_timeout and worker.busy and
                      now - worker.last_beat > self.worker_timeout):
                    reason = 'no progress for %.1f s' % (now -
                                                          worker.last_beat)
                if reason is None:
                    continue
                worker.kill_reason = reason
                logger.error('Worker %s (pid %d) presumed hung: %s; '
                             'killing it.', worker.id, worker.proc.pid,
                             reason)
                self.events.emit('worker_timeout', worker=worker.id,
                                 gpu=worker.slot.index, reason=reason)
                try:
                    worker.proc.popen.kill()
                except OSError:
                    pass

    def _reap_all(self):
        for resource in self.resources.values():
            for worker in list(resource.workers.values()):
                if worker.state == EXITED:
                    continue
                code = worker.proc.popen.poll()
                if code is None:
                    continue
                # drain remaining messages (the READY/exit of a short job)
                self._on_worker_messages(worker)
                self._on_exit(resource, worker, code)
        self._reap_standbys()

    def _reap_standbys(self):
        """Forget exited standby / retired processes (``standby_exit``
        closes their standby GPU time in the metrics).  True if a retired
        process was reaped."""
        retired = False
        for index, proc in list(self.standbys.items()):
            if proc.popen.poll() is not None:
                proc.pipe.close()
                del self.standbys[index]
                self.events.emit('standby_exit', pid=proc.pid, slot=index,
                                 code=proc.popen.returncode)
        for proc in list(self.retiring):
            if proc.popen.poll() is not None:
                proc.pipe.close()
                self.retiring.remove(proc)
                self.events.emit('standby_exit', pid=proc.pid, slot=proc.slot,
                                 code=proc.popen.returncode, retired=True)
                retired = True
        return retired

    def _on_exit(self, resource, worker, code, recycled=False):
        was_ready = worker.state in (READY, DRAINING) and worker.t_ready
        # a drained worker the watchdog had to kill still counts as failed
        drained = worker.state == DRAINING and not worker.kill_reason
        worker.state = EXITED
        worker.exit_code = code
        worker.t_exit = time.monotonic_ns()
        if not recycled:
            worker.proc.pipe.close()
        del resource.workers[worker.id]
        self.history.append(worker.summary())
        self.events.emit('worker_exit', worker=worker.id, code=code,
                         gpu=worker.slot.index, killed=worker.kill_reason,
                         recycled=recycled)
        requeued = self._requeue(resource, worker)
        if resource.kind == 'job' and code == 0 and not drained:
            resource.succeeded += 1
            resource.declared = max(0, resource.declared - 1)
        elif code != 0 and not drained:
            resource.failed += 1
            resource.consecutive_failures += 1
            delay = min(self.max_restart_backoff,
                        0.1 * (2 ** min(resource.consecutive_failures, 10)))
            resource.restart_backoff_until = time.monotonic() + delay
            logger.warning('Worker %s exited with code %s (requeued %d '
                           'items); restarting in %.1f s.', worker.id, code,
                           requeued, delay)
        if was_ready:
            resource.fence_wanted = True
        self._persist(resource)
        if self.redis is not None:
            try:
                self.redis.delete(WORKER_KEY.format(id=worker.id))
            except Exception:  # pylint: disable=broad-except
                pass

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
        if not resource.fence_wanted or not self.node.ready or \
                self.node.inflight is not None:
            return
        members = sorted((w.id for w in resource.ready()),
                         key=lambda wid: resource.workers[wid].slot.index)
        if not self.node.can_fence([resource.workers[wid].proc
                                    for wid in members]):
            return
        resource.fence_wanted = False
        if members == resource.fenced_members:
            return
        if not members:
            resource.fenced_members = []
            resource.fenced_epoch = resource.epoch
            self._publish_active(resource)
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
