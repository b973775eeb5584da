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
* **Warm pool** (:mod:`.pool`): standby processes, each pinned to its GPU
  at spawn, have imported the native kernel module (not PyTorch, unless a
  plug-in needs it), created the HIP context, loaded every code object and
  prebuilt the engine with its warm-start graph, so **a standby holds its
  GPU** (the benchmark reports this as ``standby_gpu_s``).  A scale-up
  hands a standby its assignment over a pipe, and READY is one graph
  launch.  Deep idle parks the pool when demand ends
  and wakes it, sized to the waiting keys, ahead of the tick that scales
  for them.  Standbys do not count as replicas.
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
  per GPU the communicator is persistent (:mod:`.nodecomm`, orchestrated
  by :mod:`.fencing`: built over the slots' processes, shrunk when one
  exits, regrown when one appears); otherwise each epoch bootstraps its own
  over the READY workers.  The fenced set is published
  to Redis (``kiosk:active:<ns>:<name>``).
"""
import collections
import itertools
import logging
import os
import select
import threading
import time

from ..utils.events import NULL as NULL_EVENTS
from .fencing import ACTIVE_KEY, FencingMixin  # noqa: F401
from .nodecomm import NODE_EVENTS
from .pool import POOL_KEY, SLOTS_KEY, PoolMixin  # noqa: F401
from .process import (DRAINING, EXITED, READY, STARTING,  # noqa: F401
                      ManagedProcess, Pipe, Worker, WorkerTemplate,
                      bare_worker)
from .resources import ActuatorError, ResourceList, ResourceView, \
    desired_from_body
from .state import STATE_KEY, WORKER_KEY, StateMixin  # noqa: F401

logger = logging.getLogger('GpuManager')

# pre-split names (tests, tools)
_Process, _Pipe, _bare_worker = ManagedProcess, Pipe, bare_worker
_EXIT = object()     # select() owner of a process's exit fd


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

class GpuManager(PoolMixin, FencingMixin, StateMixin):
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
                 pool_wake_lead_s=0.0, pin_mode='auto', hw_queues=0,
                 scale_policy=None):
        self.slots = list(slots)
        self.redis = redis_client
        self.state_ttl = int(state_ttl)
        self.events = events if events is not None else NULL_EVENTS
        self.max_restart_backoff = max_restart_backoff
        self.worker_timeout = float(worker_timeout or 0.0)
        self.start_timeout = float(start_timeout or 0.0)
        self.resources = collections.OrderedDict()
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
        self.history = []   # exited workers, for accounting
        # WORKER_PIN: isolate | visible | auto (isolate until a multi-rank
        # generation reports a non-xGMI peer path, then visible)
        if pin_mode not in ('isolate', 'visible', 'auto'):
            raise ValueError('WORKER_PIN must be isolate, visible or auto, '
                             'got %r' % (pin_mode,))
        self.pin_auto = pin_mode == 'auto'
        self.pin_mode = 'visible' if pin_mode == 'visible' else 'isolate'
        # WORKER_HW_QUEUES: GPU_MAX_HW_QUEUES of every process it spawns
        # (0 = leave the environment's)
        if int(hw_queues or 0) < 0 or int(hw_queues or 0) > 32:
            raise ValueError('WORKER_HW_QUEUES must be 0..32, got %r'
                             % (hw_queues,))
        self.hw_queues = int(hw_queues or 0)
        # the autoscaler's SCALE_POLICY ('reference' | 'strict'): an arrival
        # wakes a parked pool only for keys the next tick will scale for
        # (None: any arrival wakes it)
        self.wake_policy = scale_policy
        self._init_pool(pool_size, pool_template, pool_mode, recycle,
                        pool_idle_release_s, pool_wake_poll_s,
                        pool_wake_hold_s, pool_wake_lead_s, zygote)
        self._init_fencing(fence, fence_comm, fence_timeout,
                           fence_init_timeout, fence_fallback,
                           fence_fallback_after, fence_transport)

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
            patched_ns = time.monotonic_ns()
            self._reconcile(resource)
            # stamped before the reconcile, sent after it: the assignment
            # does not wait for the event sink's round trip
            self.events.emit('patch', t_ns=patched_ns, kind=kind, name=name,
                             declared=declared)
            view = resource.view()
        self._wake()
        return view

    def patch_namespaced_deployment(self, name, namespace, body):
        return self._patch('deployment', name, namespace, body)

    def patch_namespaced_job(self, name, namespace, body):
        return self._patch('job', name, namespace, body)

    def pin_fields(self):
        """The pin of a process spawned now: ``{}`` (isolate: the worker
        sets ``HIP_VISIBLE_DEVICES`` to its GPU alone) or ``{'visible':
        [every managed GPU]}`` (the worker keeps them all visible and
        selects its own in-process, ``worker/pinning.py``)."""
        if self.pin_mode != 'visible':
            return {}
        return {'visible': [s.visible_id for s in self.slots
                            if getattr(s, 'kind', 'gpu') == 'gpu' and
                            s.visible_id not in (None, '')]}

    def note_peer_path(self, gen, n, detail):
        """A multi-rank generation's RCCL reported a peer path that is not
        xGMI peer-to-peer.  With ``WORKER_PIN=auto`` the manager moves to
        the ``visible`` pin: processes spawned from now on see every managed
        GPU (RCCL may not pick P2P to a device its process cannot see), and
        idle standbys of the old pin are retired so their replacements join
        the next generation.  Called under the manager lock."""
        if not self.pin_auto or self.pin_mode == 'visible' or n < 2:
            return False
        self.pin_mode = 'visible'
        self.events.emit('pin_mode', mode='visible', reason=detail, gen=gen,
                         n=n)
        logger.warning('Generation %s (%d ranks) reported %s: spawning '
                       'workers with every managed GPU visible from now on.',
                       gen, n, detail)
        stale = [index for index, proc in self.standbys.items()
                 if getattr(proc, 'pin_mode', 'isolate') != 'visible']
        for index in stale:
            proc = self.standbys.pop(index)
            if proc.popen.poll() is None:
                proc.pipe.send({'cmd': 'exit'})
                self.retiring.append(proc)
        if stale:
            self.events.emit('standby_retired', standbys=len(stale),
                             reason='pin mode')
            self._publish_pool()
        return True

    def status(self):
        with self.lock:
            return {
                'slots': [s.to_dict() for s in self.slots],
                'standbys': [{'pid': p.pid, 'booted': p.booted,
                              'slot': index}
                             for index, p in self.standbys.items()],
                'node_comm': (self.node.summary() if self.node is not None
                              else None),
                'pin_mode': self.pin_mode,
                # deep idle: parked pool, arrival wakes, current wake lead
                'pool': {'parked': self.pool_parked,
                         'arrival_wakes': self.arrival_wakes,
                         'queue_reads': self.queue_reads,
                         'queue_reads_fine': self.queue_reads_fine,
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
                self._configure_rccl()
            with self.lock:
                self._start_zygote()
                self._refill_pool()
            self._thread = threading.Thread(target=self._loop,
                                            name='gpumgr', daemon=True)
            self._thread.start()
        return self

    def _configure_rccl(self):
        """Before the zygote and the first standby exist: point every worker
        at the one-ISA copy of RCCL (``parallel/rccl_lib.py``), so a fresh
        process's first generation does not inflate 5.3 GB of device code
        for other GPUs (1.75 s -> 0.36 s on MI355X, profiles/r5_fence_lag).
        Only for GPU slots with the RCCL transport; the fake-HIP CPU stack
        keeps its own library."""
        if os.environ.get('FENCE', 'auto') not in ('auto', 'rccl', '') or \
                self.node.transport_override not in (None, 'rccl'):
            return None
        # (traced for the fake RCCL of the CPU stack too: same log lines)
        self._configure_rccl_trace()
        ladder = [p for p in os.environ.get('KIOSK_RCCL_LADDER', '').split(
            os.pathsep) if p]
        if os.environ.get('KIOSK_NATIVE') == 'fake' or \
                not any(getattr(s, 'kind', 'gpu') == 'gpu'
                        for s in self.slots):
            # the fake-HIP CPU stack keeps its own library (a test may give
            # it a ladder of copies)
            self.node.rccl_libs = ladder
            return None
        from ..parallel import rccl_lib
        info = rccl_lib.configure(log=logger)
        if not ladder and info.get('slim') and info.get('lib'):
            # slim copy first, then the library it was made from: a slim
            # copy broken for multi-rank P2P ends on stock RCCL, not on shm
            ladder = [info['lib'], rccl_lib.source_library()]
        self.node.rccl_libs = ladder
        self.events.emit('rccl_lib', lib=info.get('lib'),
                         slim=info.get('slim'), cached=info.get('cached'),
                         ms=info.get('ms'), error=info.get('error'),
                         ladder=ladder,
                         code_object_bytes=info.get('slim_code_object_bytes'))
        return info

    def _configure_rccl_trace(self):
        """Every worker's RCCL writes its INFO log to a file of its own
        (``parallel/rccl_info.py``): its node agent reports RCCL's init
        breakdown and the transport per peer of each generation
        (``node_comm_ready`` / ``node_comm_info`` events).  The files go to
        ``RCCL_TRACE_DIR`` (kept) or a temporary directory removed at stop;
        ``RCCL_TRACE=0`` or an operator's own ``NCCL_DEBUG`` turns it off."""
        from ..parallel import rccl_info
        directory = os.environ.get('RCCL_TRACE_DIR')
        temporary = not directory
        try:
            if temporary:
                import tempfile
                directory = tempfile.mkdtemp(prefix='kiosk-rccl-')
            else:
                os.makedirs(directory, exist_ok=True)
        except OSError as err:
            logger.warning('RCCL trace directory: %s', err)
            return
        env = rccl_info.trace_env(directory)
        self.events.emit('rccl_trace', dir=directory if env else None,
                         nccl_debug=os.environ.get('NCCL_DEBUG'),
                         nccl_debug_file=os.environ.get('NCCL_DEBUG_FILE'),
                         rccl_trace=os.environ.get('RCCL_TRACE'))
        if not env:
            logger.info('RCCL INFO logs not traced (NCCL_DEBUG=%s, '
                        'NCCL_DEBUG_FILE=%s, RCCL_TRACE=%s).',
                        os.environ.get('NCCL_DEBUG'),
                        os.environ.get('NCCL_DEBUG_FILE'),
                        os.environ.get('RCCL_TRACE'))
            if temporary:
                os.rmdir(directory)
            return
        os.environ.update(env)
        self._rccl_trace_env = env        # removed again at stop
        self._rccl_trace_tmp = directory if temporary else None
        logger.info('RCCL INFO logs of every worker: %s', directory)

    def _wake(self):
        try:
            os.write(self._wake_w, b'x')
        except OSError:
            pass

    def _loop(self):
        while not self._stop.is_set():
            timeout = 0.05
            for due in (self._wake_at, self._spawn_at, self._park_at,
                        self._arrival_check_due()):
                if due is not None:
                    # a deferred arrival wake / standby spawn / queue read:
                    # do not sleep past it
                    timeout = min(timeout, max(0.001,
                                               due - time.monotonic()))
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
        for name, value in (getattr(self, '_rccl_trace_env', None) or
                            {}).items():
            if os.environ.get(name) == value:
                del os.environ[name]
        self._rccl_trace_env = None
        tmp = getattr(self, '_rccl_trace_tmp', None)
        if tmp:
            import shutil
            shutil.rmtree(tmp, ignore_errors=True)
            self._rccl_trace_tmp = None

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
            # exit fds: a reaped process closes its own, so each wakes the
            # loop once (the reap below runs on every pass)
            procs = list(self.standbys.values()) + list(self.retiring) + [
                w.proc for r in self.resources.values()
                for w in r.workers.values() if w.state != EXITED]
            for proc in procs:
                if getattr(proc, 'pidfd', None) is not None:
                    fds.setdefault(proc.pidfd, _EXIT)
        try:
            ready, _, _ = select.select(list(fds), [], [], timeout)
        except (OSError, ValueError):
            ready = []
        with self.lock:
            for fd in ready:
                owner = fds.get(fd)
                if owner is _EXIT:
                    continue              # reaped below
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
            self._reap_orphans()
            self._watchdog()
            if self.zygote_enabled and not self._check_zygote():
                self._start_zygote()      # a dead zygote, after a pause
            if self.node is not None and not self._stopping:
                self.node.step()
            for resource in self.resources.values():
                self._reconcile(resource)
                self._maybe_fence(resource)
            self._refill_pool()

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
        assign.update(self.pin_fields())
        proc = self._take_standby(resource.template, slot)
        from_pool = proc is not None
        sizing = None
        if from_pool and proc.hbm_free:
            sizing = self._size_from_free(resource, assign, proc.hbm_free,
                                          slot)
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
        if sizing is not None:
            self.events.emit('hbm_sizing', **sizing)
        self.events.emit('worker_assigned', worker=wid, gpu=slot.index,
                         pid=proc.pid, from_pool=from_pool,
                         resource=resource.name)
        logger.info('Started worker %s on GPU %s (pid %d, %s).', wid,
                    slot.visible_id or slot.index, proc.pid,
                    'warm pool' if from_pool else 'cold spawn')
        return worker

    def _size_from_free(self, resource, assign, free, slot):
        """N5: clamp this assignment's KEYS_PER_POD (the job worker's batch)
        to what fits in the HBM the standby measured free.  Returns the
        ``hbm_sizing`` event's fields."""
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
        # the event's fields: sent once the assignment is on its way
        return {'t_ns': time.monotonic_ns(), 'gpu': slot.index,
                'hbm_free': free, 'max_keys_per_pod': limit,
                'keys_per_pod': kpp, 'requested': tpl.keys_per_pod}

    def _drain(self, worker, reason, recycle=None):
        if worker.state in (DRAINING, EXITED):
            return
        worker.state = DRAINING
        if recycle is None:
            recycle = self._recycle_ok(worker.resource)
        worker.proc.pipe.send({'cmd': 'drain', 'reason': reason,
                               'recycle': bool(recycle)})
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
                            and worker.t_ready and \
                            worker.quarantined_at is None:
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
            elif kind == 'pull_error':
                # the worker stays up and retries; surfaced once per burst
                worker.pull_errors += 1
                if worker.pull_errors in (1, 10, 100):
                    logger.error('Worker %s cannot pull keys (%d errors): %s',
                                 worker.id, worker.pull_errors,
                                 message.get('message'))
                    self.events.emit('worker_pull_error', worker=worker.id,
                                     errors=worker.pull_errors,
                                     message=message.get('message'))
    # a quarantined worker (its node agent stopped answering) that holds no
    # key and has not exited this long after the drain is hung as a whole:
    # killed (a busy one is the WORKER_TIMEOUT watchdog's)
    QUARANTINE_EXIT_S = 30.0

    def _watchdog(self):
        """Failure detection beyond waitpid: kill workers that
        are alive but stuck.  The kill is an ordinary death afterwards --
        reaped, items requeued, restart backoff, fence re-run."""
        now = time.monotonic()
        for resource in self.resources.values():
            for worker in resource.workers.values():
                if worker.state == EXITED or worker.kill_reason:
                    continue
                reason = None
                if worker.quarantined_at is not None and not worker.busy \
                        and now - max(worker.quarantined_at, worker.last_beat) > \
                        self.QUARANTINE_EXIT_S:
                    reason = 'quarantined and silent for %.0f s' % (
                        now - max(worker.quarantined_at, worker.last_beat))
                elif (self.start_timeout and worker.state == STARTING and
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

    def _on_exit(self, resource, worker, code, recycled=False):
        was_ready = worker.state in (READY, DRAINING) and worker.t_ready
        # a drained worker the watchdog had to kill still counts as failed
        drained = worker.state == DRAINING and not worker.kill_reason
        worker.state = EXITED
        worker.exit_code = code
        worker.t_exit = time.monotonic_ns()
        if not recycled:
            worker.proc.close()
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
