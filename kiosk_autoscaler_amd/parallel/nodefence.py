"""Persistent node-wide membership communicator (SURVEY N4, round-2 design).

Round 1 re-bootstrapped an RCCL communicator over the READY workers at every
membership change (~250 ms of ``ncclCommInitRank`` per scale event at one
rank, more at eight).  But the processes behind the GPU slots are long-lived:
a standby becomes a worker, a drained worker is recycled back into its
GPU's standby, and the process (HIP context, RCCL state) survives both.  So
the communicator is built **once** over every slot's process and every
membership change is fenced by the 72-byte all-reduce alone:

* ``comm_init {gen, rank, nranks}`` -- rank 0 (lowest slot) creates the
  communicator id and reports it (``comm_uid``); the manager relays it to the
  other ranks; all connect.  Each rank reports ``comm_ready``.  This happens
  at pool boot and again only after a slot's process *dies* (no grow in
  RCCL, so a replacement process means a new generation).
* ``fence {epoch, gen, slots}`` -- every rank contributes
  ``{epoch, bit(own slot in slots)}`` to the int64[1 + 8] sum; standbys and
  other resources' workers contribute zeros.  The result must equal
  ``{epoch * nranks, membership mask}``; rank 0 acknowledges (``fenced``).
* ``comm_shrink {gen, sub, excluded}`` -- a slot's process died or retired:
  the survivors drop its rank (``ncclCommShrink`` with
  ``NCCL_SHRINK_ABORT``: an all-reduce blocked on the dead peer is first
  *interrupted* -- ``Fence::request_interrupt`` from the reader thread, the
  communicator is kept -- then terminated by the shrink) and keep fencing
  with that slot's bit at 0 while its replacement boots; the manager starts
  the next full generation once every slot has a live process again.
* ``comm_abort {gen}`` -- the generation is dropped: any blocked collective
  is aborted (``Fence::request_abort`` is safe from the reader thread).

Transports: :class:`RcclNodeTransport` (production, RCCL over xGMI through
``_kiosk_hip.Fence``), :class:`ShmNodeTransport` (production when the
standbys hold no GPU, and the default fallback: a native host shared-memory
all-reduce, ``_kiosk_hip.ShmComm``), :class:`GlooNodeTransport` (CPU test
fake, one persistent gloo group per generation, cannot shrink) and
:class:`StoreNodeTransport` (Redis lists; mock CPU workers).
"""
import json
import logging
import os
import queue
import tempfile
import threading
import time
import uuid

from .fence import MIN_SLOTS, FenceError

logger = logging.getLogger('NodeFence')

NODE_COMMANDS = ('comm_init', 'comm_uid', 'comm_shrink', 'comm_abort', 'fence',
                 'fence_abort', 'fence_commit')
NODE_EVENTS = ('comm_uid', 'comm_ready', 'fenced', 'node_agent',
               'node_preloaded', 'comm_info')
STORE_KEY = 'kiosk:nodefence:{uid}:{epoch}'


def node_vector(epoch, slot, member_slots, width):
    vec = [0] * (1 + width)
    vec[0] = int(epoch)
    if int(slot) in set(int(s) for s in member_slots):
        vec[1 + int(slot)] = 1
    return vec


def node_expected(epoch, nranks, member_slots, width):
    vec = [0] * (1 + width)
    vec[0] = int(epoch) * int(nranks)
    for slot in member_slots:
        vec[1 + int(slot)] += 1
    return vec


def node_width(slot_count):
    return max(MIN_SLOTS, int(slot_count))


class FenceInterrupted(FenceError):
    """A collective given up because the manager is shrinking a rank out:
    the communicator is still usable for the shrink (not dropped)."""


def _survivor_rank(rank, excluded):
    return rank - sum(1 for r in excluded if int(r) < rank)


# RCCL's per-process init started at process start (start_early_preload)
_EARLY = {}


def start_early_preload(native=None):
    """Start RCCL's per-process one-time init -- ``ncclGetVersion`` +
    ``ncclGetUniqueId``: the library's init and its bootstrap network,
    ~120 ms -- on a thread of its own as the process starts, in parallel with
    the HIP context and the engine build, instead of after them on the node
    agent's thread, where it delayed every woken worker's first generation
    (profiles/r5_fence_lag).  No kernel is loaded here: RCCL's code-object
    load stays in the generation's init, after READY.  The agent's
    :meth:`RcclNodeTransport.preload` joins this thread."""
    if 'thread' in _EARLY or not _rccl_mapped():
        # (not mapped: a cold-spawned worker, whose first RCCL call would
        # also register RCCL's fat binary -- seconds under the runtime lock
        # every kernel launch waits on, profiles/r4_collision -- in the
        # middle of its engine build; its agent loads RCCL after the build)
        return

    def run():
        t0 = time.perf_counter()
        try:
            mod = native
            if mod is None:
                from ..ops import native as native_ops
                mod = native_ops.load()
            mod.fence_preload()
            _EARLY['ms'] = (time.perf_counter() - t0) * 1e3
        except Exception as err:  # pylint: disable=broad-except
            _EARLY['error'] = err

    thread = threading.Thread(target=run, name='rccl-preload', daemon=True)
    _EARLY['thread'] = thread
    thread.start()


def _rccl_mapped():
    """RCCL is already mapped -- and its fat binary registered -- in this
    process (the zygote dlopens it before forking)."""
    try:
        with open('/proc/self/maps') as maps:
            return any('librccl' in line or 'fake_hip_rccl' in line
                       for line in maps)
    except OSError:
        return False


# ---------------------------------------------------------------------------
# transports: make_uid (rank 0) / connect (collective) / allreduce / abort
# ---------------------------------------------------------------------------
class RcclNodeTransport(object):
    name = 'rccl'

    def __init__(self, timeout=60.0, native=None, trace=None):
        if native is None:
            from ..ops import native as native_ops
            native = native_ops.load()
        self.native = native
        self.timeout = float(timeout)
        self.comm = None
        # this process's RCCL INFO log, when the manager routed it to a
        # file (parallel/rccl_info.py): init breakdown, peer transports
        if trace is None:
            from .rccl_info import RcclTrace
            trace = RcclTrace.for_process()
        self.trace = trace

    def info(self):
        """What RCCL logged since the last call (parsed), or None."""
        if self.trace is None:
            return None
        from .rccl_info import summary
        parsed = self.trace.take()
        return summary(parsed) if parsed is not None else None

    def preload(self):
        """RCCL's per-process one-time costs (library load + init), paid
        when the agent starts rather than inside a generation: ms."""
        early = _EARLY.get('thread')
        if early is not None:
            early.join()
            if 'error' in _EARLY:
                raise _EARLY['error']
            return _EARLY.get('ms', 0.0)
        preload = getattr(self.native, 'fence_preload', None)
        return preload() if preload is not None else 0.0

    def use_library(self, lib):
        """Make ``lib`` the RCCL this process's next communicator uses
        (the manager's library ladder, gpumgr/nodecomm.py); loaded beside
        any other already mapped.  Returns the library in use."""
        use = getattr(self.native, 'fence_use_library', None)
        if use is None:
            return None
        return use(lib or '')

    @property
    def library(self):
        try:
            return self.native.rccl_library()
        except Exception:  # pylint: disable=broad-except
            return None

    def make_uid(self, gen, lib=None):
        if lib:
            self.use_library(lib)
        return self.native.fence_unique_id().hex()

    def connect(self, gen, rank, nranks, uid, should_abort=None,
                timeout=None, lib=None):
        # two-phase: the object exists before the collective blocks, so a
        # peer death can abort it from the reader thread (request_abort);
        # an abort that raced ahead of the assignment is caught by the
        # check right after it.  ``timeout``: this connect's bound (a
        # first generation's is longer); collectives keep ``self.timeout``
        if lib:
            self.use_library(lib)
        self.comm = self.native.Fence(nranks, rank, timeout or self.timeout)
        if should_abort is not None and should_abort():
            self.comm.request_abort()
        self.comm.connect(bytes.fromhex(uid))
        if timeout and hasattr(self.comm, 'set_timeout'):
            self.comm.set_timeout(self.timeout)

    @property
    def can_shrink(self):
        try:
            return bool(self.native.fence_can_shrink())
        except Exception:  # pylint: disable=broad-except
            return False

    def allreduce(self, epoch, vec):
        interrupted = getattr(self.native, 'FenceInterrupted', None)
        try:
            result, us = self.comm.allreduce(list(vec))
        except Exception as err:
            if interrupted is not None and isinstance(err, interrupted):
                raise FenceInterrupted(str(err))
            raise
        return list(result), {'allreduce_us': us}

    def request_interrupt(self):
        comm = self.comm
        if comm is not None:
            comm.request_interrupt()

    def shrink(self, excluded, timeout=None):
        """Survivors only: ``ncclCommShrink(NCCL_SHRINK_ABORT)``."""
        if self.comm is None:
            raise FenceError('no communicator to shrink')
        self.comm.shrink([int(r) for r in excluded],
                         self.timeout if timeout is None else timeout, True)

    def request_abort(self):
        comm = self.comm
        if comm is not None:
            comm.request_abort()

    def close(self):
        comm, self.comm = self.comm, None
        if comm is not None:
            try:
                comm.destroy()   # aborts instead when an abort was requested
            except Exception:  # pylint: disable=broad-except
                pass


class ShmNodeTransport(object):
    """Native host shared-memory all-reduce (``_kiosk_hip.ShmComm``): the
    node communicator of the pool modes whose standbys hold no GPU
    (``context`` / ``import`` / deep idle) -- an RCCL communicator would
    need a hardware queue and ~0.8 GiB of HBM per GPU to agree on 9
    integers -- and the fallback when RCCL cannot build one.  Notices a dead
    peer by itself (its pid), which RCCL does not."""

    name = 'shm'
    can_shrink = True

    def __init__(self, timeout=30.0, native=None, shm_dir=''):
        if native is None:
            from ..ops import native as native_ops
            native = native_ops.load(torch_first=False)
        self.native = native
        self.timeout = float(timeout)
        self.shm_dir = shm_dir or os.environ.get('KIOSK_SHM_DIR', '')
        self.comm = None
        self._interrupt = False

    def make_uid(self, gen):
        return self.native.shm_unique_id(self.shm_dir)

    def connect(self, gen, rank, nranks, uid, should_abort=None,
                timeout=None):
        self._interrupt = False
        self.comm = self.native.ShmComm(uid, nranks, rank, self.timeout)
        if should_abort is not None and should_abort():
            self.comm.request_abort()
        self.comm.wait_ready()

    def allreduce(self, epoch, vec):
        try:
            result, us = self.comm.allreduce(list(vec))
        except RuntimeError as err:
            text = str(err)
            # a peer that died / left, or the manager's interrupt: the
            # communicator itself is fine, the survivors shrink it
            if self._interrupt or 'died' in text or 'left' in text:
                raise FenceInterrupted(text)
            raise
        return list(result), {'allreduce_us': us}

    def request_interrupt(self):
        self._interrupt = True
        comm = self.comm
        if comm is not None:
            comm.request_abort()   # per object: the shrunk child is fresh

    def shrink(self, excluded, timeout=None):
        if self.comm is None:
            raise FenceError('no communicator to shrink')
        child = self.comm.shrink([int(r) for r in excluded])
        self.comm.close()
        self.comm = child
        self._interrupt = False
        child.wait_ready()

    def request_abort(self):
        comm = self.comm
        if comm is not None:
            comm.request_abort()

    def close(self):
        comm, self.comm = self.comm, None
        if comm is not None:
            comm.close()


def sweep_stale_shm(dirs=None, older_than=300.0, now=None):
    """Remove ``kiosk-shm-*`` segments left behind by generations whose
    ranks all died before joining (a joined generation unlinks its file at
    once, so nothing live is older than its ``FENCE_INIT_TIMEOUT``).  The
    manager calls it at start; returns the paths removed."""
    now = time.time() if now is None else now
    if dirs is None:
        dirs = (os.environ.get('KIOSK_SHM_DIR') or '/dev/shm', '/tmp')
    removed = []
    for directory in dirs:
        try:
            names = os.listdir(directory)
        except OSError:
            continue
        for name in names:
            if not name.startswith('kiosk-shm-'):
                continue
            path = os.path.join(directory, name)
            try:
                if now - os.stat(path).st_mtime < older_than:
                    continue
                os.unlink(path)
                removed.append(path)
            except OSError:
                pass
    return removed


class GlooNodeTransport(object):
    """One persistent gloo group per generation over a FileStore (CPU)."""

    name = 'gloo'

    def __init__(self, timeout=30.0, root=None):
        self.timeout = float(timeout)
        self.root = root or tempfile.gettempdir()
        self.pg = None
        self._aborted = False

    def make_uid(self, gen):
        return os.path.join(self.root, 'kiosk-nodefence-%d-%s' % (
            gen, uuid.uuid4().hex[:12]))

    def connect(self, gen, rank, nranks, uid, should_abort=None,
                timeout=None):
        import datetime
        import torch.distributed as dist
        self._aborted = bool(should_abort and should_abort())
        store = dist.FileStore(uid, nranks)
        self.pg = dist.ProcessGroupGloo(
            store, rank, nranks, datetime.timedelta(seconds=self.timeout))

    def allreduce(self, epoch, vec):
        import torch
        if self._aborted:
            raise FenceError('communicator aborted')
        tensor = torch.tensor(vec, dtype=torch.int64)
        t0 = time.perf_counter()
        self.pg.allreduce([tensor]).wait()
        return tensor.tolist(), {'allreduce_us': (time.perf_counter() - t0)
                                 * 1e6}

    can_shrink = False

    def request_abort(self):
        self._aborted = True   # gloo cannot be interrupted: its timeout ends it

    def request_interrupt(self):
        pass

    def shrink(self, excluded, timeout=None):
        raise FenceError('a gloo group cannot shrink')

    def close(self):
        self.pg = None


class StoreNodeTransport(object):
    """All-reduce through Redis lists (every rank sums every vector)."""

    name = 'store'

    def __init__(self, redis=None, timeout=30.0):
        self._redis = redis
        self.timeout = float(timeout)
        self.uid = None
        self.nranks = 0
        self.rank = 0
        self._aborted = False
        self._interrupt = False
        self._shrinks = 0

    can_shrink = True

    @property
    def redis(self):
        if self._redis is None:
            from ..redisq import StrictRedis
            self._redis = StrictRedis(
                host=os.environ.get('REDIS_HOST', '127.0.0.1'),
                port=int(os.environ.get('REDIS_PORT', 6379)),
                decode_responses=True)
        return self._redis

    def make_uid(self, gen):
        return '%d-%s' % (gen, uuid.uuid4().hex[:12])

    def connect(self, gen, rank, nranks, uid, should_abort=None,
                timeout=None):
        self.uid, self.rank, self.nranks = uid, rank, nranks
        self._aborted = bool(should_abort and should_abort())
        self._interrupt = False
        self._shrinks = 0

    def allreduce(self, epoch, vec):
        key = STORE_KEY.format(uid=self.uid, epoch=epoch)
        t0 = time.perf_counter()
        self.redis.rpush(key, json.dumps([self.rank, vec]))
        if self.rank == 0:
            self.redis.expire(key, 120)
        deadline = time.monotonic() + self.timeout
        while True:
            entries = self.redis.lrange(key, 0, -1)
            if len(set(json.loads(e)[0] for e in entries)) >= self.nranks:
                break
            if self._interrupt:
                raise FenceInterrupted('store all-reduce interrupted')
            if self._aborted:
                raise FenceError('communicator aborted')
            if time.monotonic() > deadline:
                raise FenceError('store all-reduce epoch %s timed out (%d/%d)'
                                 % (epoch, len(entries), self.nranks))
            time.sleep(0.001)
        total = [0] * len(vec)
        seen = set()
        for entry in entries:
            rank, values = json.loads(entry)
            if rank in seen:
                continue
            seen.add(rank)
            total = [a + b for a, b in zip(total, values)]
        return total, {'allreduce_us': (time.perf_counter() - t0) * 1e6}

    def request_interrupt(self):
        self._interrupt = True

    def shrink(self, excluded, timeout=None):
        if self.uid is None:
            raise FenceError('no communicator to shrink')
        self._shrinks += 1
        self.uid = '%s.s%d' % (self.uid.split('.s')[0], self._shrinks)
        self.rank = _survivor_rank(self.rank, excluded)
        self.nranks -= len(excluded)
        self._interrupt = False

    def request_abort(self):
        self._aborted = True

    def close(self):
        self.uid = None


def init_timeout(default=12.0):
    """``FENCE_INIT_TIMEOUT``: seconds a node-communicator generation may
    take to connect (and an all-reduce to complete) before it is failed."""
    try:
        return float(os.environ.get('FENCE_INIT_TIMEOUT', default))
    except ValueError:
        return default


def choose_node_transport(kind, backend, timeout=None):
    timeout = init_timeout() if timeout is None else float(timeout)
    if kind in ('auto', ''):
        kind = 'rccl' if backend == 'hip' else 'store'
    if kind == 'rccl':
        return RcclNodeTransport(timeout)
    if kind == 'shm':
        return ShmNodeTransport(timeout)
    if kind == 'gloo':
        return GlooNodeTransport(min(timeout, 30.0))
    if kind == 'store':
        return StoreNodeTransport(timeout=min(timeout, 30.0))
    raise ValueError('unknown FENCE transport %r' % kind)


# ---------------------------------------------------------------------------
# per-process agent
# ---------------------------------------------------------------------------
class NodeFenceAgent(object):
    """Lives as long as the process (standby and worker phases alike) and
    runs node-communicator commands in order on one thread.

    ``idle`` is cleared while a collective is in flight: the serving loop
    chunks its forward passes (FENCE_YIELD_CHUNK_MS) so the all-reduce
    kernel is not queued behind a whole key of GEMMs."""

    def __init__(self, slot, transport, channel=None, events=None,
                 uid_timeout=None, transport_factory=None, preload=False):
        self.slot = int(slot)
        self.transport = transport
        # the configured transport: a generation that names none (the RCCL
        # retry after a fallback, gpumgr/nodecomm.py) goes back to it
        self.home_transport = transport
        # kind -> transport, for a manager-requested switch (the fallback
        # after failed RCCL generations, gpumgr/nodecomm.py)
        self.transport_factory = transport_factory or (
            lambda kind: choose_node_transport(kind, 'hip'))
        self.channel = channel
        self.events = events
        self.uid_timeout = float(init_timeout() if uid_timeout is None
                                 else uid_timeout)
        self.gen = 0          # generation of the connected communicator
        self.sub = 0          # shrinks applied to it
        self.rank = None
        self.nranks = 0
        # group -> (seq, epoch, mask): the last membership this rank agreed
        # on per resource -- its own all-reduce result, once the manager
        # committed that fence (``fence_commit``: a fence the manager
        # cancelled, e.g. before a shrink, never gates anything).
        # The worker gates its queue pulls on it (worker/runtime.py)
        self.agreed = {}
        self._results = {}    # seq -> (group, agreement) awaiting a commit
        # seqs the manager committed before this rank stored their result:
        # a commit can overtake the rank's own result (the reader thread
        # handles ``fence_commit`` as soon as rank 0's report went out;
        # ADVICE r4), so a result stored after its commit is promoted at once
        self._early_commits = set()
        self.agreed_cv = threading.Condition()
        self._uids = {}
        self._uid_cv = threading.Condition()
        self._abort_gen = 0   # highest generation the manager aborted
        self._aborted_epochs = set()
        self._queue = queue.Queue()
        self.completed = []
        self.idle = threading.Event()
        self.idle.set()
        self._freeze_ms = 0.0    # fault injection (utils/faults.py)
        self.preload_ms = None
        self._thread = threading.Thread(target=self._run, name='nodefence',
                                        daemon=True)
        if preload and hasattr(self.transport, 'preload'):
            # RCCL's one-time load, first thing on the agent thread.  It
            # holds the HIP runtime lock every kernel launch of the process
            # waits on (profiles/r4_collision); the standby built its engine
            # before this agent started, so its READY is graph launches that
            # never wait, and a first generation then connects without
            # paying the load inside its timeout
            self._queue.put({'cmd': '_preload'})
        self._thread.start()

    # -- reader-thread side ------------------------------------------------
    def submit(self, message):
        cmd = message.get('cmd')
        if cmd == 'comm_uid':
            with self._uid_cv:
                self._uids[int(message['gen'])] = message['uid']
                self._uid_cv.notify_all()
            return
        if cmd == 'fence_abort':
            self._aborted_epochs.add(message.get('seq'))
            return
        if cmd == 'fence_commit':
            self._commit(int(message.get('seq', 0)))
            return
        if cmd == 'comm_shrink':
            # a collective blocked on the dead peer gives up now -- without
            # dropping the communicator the shrink needs
            if int(message.get('gen', 0)) == self.gen:
                interrupt = getattr(self.transport, 'request_interrupt', None)
                if interrupt is not None:
                    interrupt()
        if cmd == 'comm_abort':
            gen = int(message.get('gen', 0))
            with self._uid_cv:
                self._abort_gen = max(self._abort_gen, gen)
                self._uid_cv.notify_all()
            if gen >= self.gen:   # never the comm of a newer generation
                self.transport.request_abort()
        self._queue.put(message)

    def _aborted(self, gen):
        return self._abort_gen >= gen

    def freeze_next_fence(self, ms):
        """Fault injection (``freeze_agent``): the agent thread stalls this
        long before its next fence, as a wedged rank would."""
        self._freeze_ms = float(ms)

    # -- agent thread ------------------------------------------------------
    def _emit(self, ev, **fields):
        if self.channel is not None:
            self.channel.emit(ev, **fields)

    def _preload(self):
        t0 = time.perf_counter()
        try:
            self.transport.preload()
            self.preload_ms = (time.perf_counter() - t0) * 1e3
            self._emit('node_preloaded', ms=self.preload_ms,
                       transport=self.transport.name)
        except Exception as err:  # pylint: disable=broad-except
            logger.warning('RCCL preload failed: %s', err)
            self._emit('node_preloaded', ms=None, error=str(err),
                       transport=self.transport.name)

    def _wait_uid(self, gen, timeout=None):
        deadline = time.monotonic() + (timeout or self.uid_timeout)
        with self._uid_cv:
            while gen not in self._uids:
                if self._aborted(gen):
                    raise FenceError('generation %d aborted' % gen)
                left = deadline - time.monotonic()
                if left <= 0:
                    raise FenceError('no communicator id for generation %d'
                                     % gen)
                self._uid_cv.wait(min(left, 0.5))
            return self._uids.pop(gen)

    def _comm_init(self, message):
        gen, rank = int(message['gen']), int(message['rank'])
        nranks = int(message['nranks'])
        # a generation with a process that never connected over RCCL gets
        # the manager's longer first-generation budget
        timeout = float(message.get('timeout') or 0.0) or None
        self._drop()
        wanted = message.get('transport')
        if not wanted:
            # no override: the configured transport, also after a fallback
            self.transport = self.home_transport
        elif wanted != self.transport.name:
            try:
                self.transport = self.transport_factory(wanted)
            except Exception as err:  # pylint: disable=broad-except
                logger.warning('cannot switch to transport %s: %s', wanted,
                               err)
        t0 = time.perf_counter()
        try:
            if self._aborted(gen):
                raise FenceError('generation %d aborted' % gen)
            lib = message.get('lib') if self.transport.name == 'rccl' \
                else None
            if rank == 0:
                uid = (self.transport.make_uid(gen, lib=lib) if lib else
                       self.transport.make_uid(gen))
                self._emit('comm_uid', gen=gen, uid=uid)
            else:
                uid = self._wait_uid(gen, timeout)
            extra = {'timeout': timeout} if timeout else {}
            if lib:
                extra['lib'] = lib
            self.transport.connect(gen, rank, nranks, uid,
                                   should_abort=lambda: self._aborted(gen),
                                   **extra)
        except Exception as err:  # pylint: disable=broad-except
            logger.warning('communicator generation %d failed: %s', gen, err)
            self._drop()
            self._emit('comm_ready', gen=gen, rank=rank, ok=False,
                       detail=str(err), transport=self.transport.name)
            return
        self.gen, self.rank, self.nranks, self.sub = gen, rank, nranks, 0
        init_ms = (time.perf_counter() - t0) * 1e3
        extra = {}
        info = self._rccl_info()
        if info:
            extra['rccl'] = info
        self._init_info = info or {}
        # the peer transports are known after the first collective (RCCL
        # connects lazily): reported then, once per generation
        self._info_due = (gen, 0)
        library = getattr(self.transport, 'library', None)
        if library:
            extra['lib'] = library
        self._emit('comm_ready', gen=gen, rank=rank, ok=True, init_ms=init_ms,
                   transport=self.transport.name, n=nranks, sub=0,
                   mode='init',
                   can_shrink=bool(getattr(self.transport, 'can_shrink',
                                           False)), **extra)

    def _comm_shrink(self, message):
        gen, sub = int(message['gen']), int(message['sub'])
        excluded = [int(r) for r in message.get('excluded', [])]
        t0 = time.perf_counter()
        try:
            if self.rank is None or gen != self.gen or sub != self.sub + 1:
                raise FenceError('cannot shrink generation %d.%d (have %s)'
                                 % (gen, sub, '%d.%d' % (self.gen, self.sub)
                                    if self.rank is not None else 'none'))
            if self.rank in excluded:
                raise FenceError('rank %d is excluded' % self.rank)
            self.transport.shrink(excluded)
        except Exception as err:  # pylint: disable=broad-except
            logger.warning('shrink of generation %d failed: %s', gen, err)
            rank = self.rank
            self._drop()
            self._emit('comm_ready', gen=gen, sub=sub, rank=rank, ok=False,
                       detail=str(err), transport=self.transport.name,
                       mode='shrink')
            return
        self.rank = _survivor_rank(self.rank, excluded)
        self.nranks -= len(excluded)
        self.sub = sub
        self._emit('comm_ready', gen=gen, sub=sub, rank=self.rank, ok=True,
                   init_ms=(time.perf_counter() - t0) * 1e3,
                   transport=self.transport.name, n=self.nranks,
                   mode='shrink', can_shrink=True)

    def _rccl_info(self):
        hook = getattr(self.transport, 'info', None)
        if not callable(hook):
            return None
        try:
            return hook()
        except Exception:  # pylint: disable=broad-except
            return None

    def _report_connections(self, report):
        """After a generation's first successful all-reduce: what RCCL
        connected (transport per peer, link types), to the manager."""
        due = getattr(self, '_info_due', None)
        if due is None or due != (report.get('gen'), report.get('sub', 0)):
            return
        self._info_due = None
        info = self._rccl_info()
        if info is None:
            return
        # the graph link types are logged at init, the connections now
        init = getattr(self, '_init_info', None) or {}
        links = list(init.get('link_types') or [])
        links += [t for t in info.get('link_types') or () if t not in links]
        if links:
            info['link_types'] = links
        if info.get('memory_bytes') is None and init.get('memory_bytes'):
            info['memory_bytes'] = init['memory_bytes']
        self._emit('comm_info', gen=report.get('gen'),
                   sub=report.get('sub', 0), rank=report.get('rank'),
                   n=report.get('n'), rccl=info,
                   allreduce_us=report.get('allreduce_us'))

    def _drop(self):
        self.transport.close()
        self.rank = None
        self.nranks = 0
        self.sub = 0

    def run_fence(self, message):
        epoch = int(message['epoch'])
        gen = int(message['gen'])
        sub = int(message.get('sub', 0))
        members = [int(s) for s in message.get('slots', [])]
        width = node_width(message.get('width', MIN_SLOTS))
        if self.rank is None or gen != self.gen or sub != self.sub:
            raise FenceError('no communicator for generation %d.%d (have %s)'
                             % (gen, sub, '%d.%d' % (self.gen, self.sub)
                                if self.rank is not None else 'none'))
        vec = node_vector(epoch, self.slot, members, width)
        t0 = time.perf_counter()
        # node-wide sequence number: epochs are per resource
        result, info = self.transport.allreduce(message.get('seq', epoch),
                                                vec)
        wall_ms = (time.perf_counter() - t0) * 1e3
        expected = node_expected(epoch, self.nranks, members, width)
        ok = list(result) == expected
        report = {'epoch': epoch, 'seq': message.get('seq'), 'gen': gen,
                  'sub': sub, 'ok': ok, 'rank': self.rank,
                  'n': self.nranks, 'transport': self.transport.name,
                  'wall_ms': wall_ms, 'init_ms': 0.0,
                  'mode': 'shrink' if sub else 'node'}
        report.update(info)
        if ok:
            # the agreed membership, read from this rank's own result
            mask = [i for i, bit in enumerate(result[1:]) if bit]
            seq = int(message.get('seq', 0))
            entry = (message.get('group'), {'seq': seq, 'epoch': epoch,
                                            'slots': mask})
            with self.agreed_cv:
                if seq in self._early_commits:
                    # the commit arrived first: this result is published
                    self._early_commits.discard(seq)
                    self._promote(entry)
                else:
                    self._results[seq] = entry
        else:
            report['detail'] = 'got %s expected %s' % (result, expected)
        return report

    def _commit(self, seq):
        """The manager published fence ``seq``: its result becomes this
        rank's agreed membership (results of older fences are dropped)."""
        with self.agreed_cv:
            entry = self._results.pop(seq, None)
            for old in [k for k in self._results if k < seq]:
                del self._results[old]
            if entry is not None:
                self._promote(entry)
                return
            self._early_commits.add(seq)
            # bounded: a commit whose result never comes (a fence this rank
            # skipped) is forgotten once much newer ones exist
            for old in [k for k in self._early_commits if k < seq - 64]:
                self._early_commits.discard(old)

    def _promote(self, entry):
        """(under ``agreed_cv``) a committed result becomes the group's
        agreed membership unless a newer one already is."""
        group, agreement = entry
        current = self.agreed.get(group)
        if current is None or current['seq'] < agreement['seq']:
            self.agreed[group] = agreement
            self.agreed_cv.notify_all()

    def agreement(self, group):
        """``{'seq', 'epoch', 'slots'}`` of the last fence of ``group`` this
        rank completed, or None."""
        with self.agreed_cv:
            return self.agreed.get(group)

    def _run(self):
        while True:
            message = self._queue.get()
            if message is None:
                return
            cmd = message.get('cmd')
            if cmd == '_preload':
                self._preload()
                continue
            if cmd == 'comm_init':
                self._comm_init(message)
                continue
            if cmd == 'comm_shrink':
                self._comm_shrink(message)
                continue
            if cmd == 'comm_abort':
                if int(message.get('gen', 0)) >= self.gen:
                    self._drop()
                continue
            if cmd != 'fence':
                continue
            epoch = message.get('epoch')
            if message.get('seq') in self._aborted_epochs:
                continue
            if self._freeze_ms > 0:
                freeze, self._freeze_ms = self._freeze_ms, 0.0
                logger.warning('fault: node agent frozen for %.0f ms', freeze)
                time.sleep(freeze / 1e3)
            self.idle.clear()
            try:
                report = self.run_fence(message)
            except Exception as err:  # pylint: disable=broad-except
                logger.warning('node fence epoch %s failed: %s', epoch, err)
                report = {'epoch': epoch, 'seq': message.get('seq'),
                          'gen': message.get('gen'),
                          'ok': False, 'detail': str(err), 'rank': self.rank,
                          'transport': self.transport.name, 'mode': 'node',
                          'interrupted': isinstance(err, FenceInterrupted)}
                if not isinstance(err, FenceInterrupted):
                    self._drop()   # a failed collective leaves no usable comm
            finally:
                self.idle.set()
            self.completed.append(report)
            if report.get('ok'):
                self._report_connections(report)
            if self.events is not None:
                self.events.emit('fence_rank', slot=self.slot, **report)
            if report.get('rank') == 0 or not report['ok']:
                self._emit('fenced', **report)

    def close(self, timeout=5.0):
        self._queue.put(None)
        self._thread.join(timeout=timeout)
        if self._thread.is_alive():
            return False
        self._drop()
        return True
