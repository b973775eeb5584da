"""Membership fence: every READY worker agrees on the active set.

The reference has no consistency mechanism beyond "Kubernetes owns it"
(SURVEY §5.8).  Here every change of the READY worker set starts a fence
*epoch* (issued by the GPU manager, coalesced, one in flight):

1. rank 0 of the new member list creates the communicator id and publishes
   it through Redis (``kiosk:fence:<group>:<epoch>:uid``); the others read it.
2. the members build (or shrink) their communicator and all-reduce the
   72-byte ``int64[1 + 8]`` vector ``{epoch, one bit per GPU slot}``
   (sum).  The result must equal ``{epoch * n, expected membership}``.
3. rank 0 acknowledges to the manager, which then publishes the set.

Transports (same protocol, different collective):

* :class:`RcclTransport` -- production: RCCL over xGMI through the native
  module (``ncclCommInitRank`` for a new set; ``ncclCommShrink`` when the
  new set is a subset of the current communicator, so a scale-down costs no
  re-bootstrap; ``ncclCommAbort`` on timeout).
* :class:`GlooTransport` -- CPU test fake: a per-epoch gloo process group
  over a node-local ``FileStore`` (multi-process tests without a GPU).
* :class:`StoreTransport` -- Redis-only fallback (mock CPU workers).

The payload is latency-bound (72 B): RCCL picks its small-message
algorithm; xGMI bandwidth is irrelevant here.
"""
import json
import logging
import os
import queue
import tempfile
import threading
import time

logger = logging.getLogger('Fence')

UID_KEY = 'kiosk:fence:{group}:{epoch}:uid'
STORE_KEY = 'kiosk:fence:{group}:{epoch}:vec'
MIN_SLOTS = 8


def build_vector(epoch, slot, width):
    vec = [0] * (1 + width)
    vec[0] = int(epoch)
    vec[1 + int(slot)] = 1
    return vec


def expected_vector(epoch, slots, width):
    vec = [0] * (1 + width)
    vec[0] = int(epoch) * len(slots)
    for slot in slots:
        vec[1 + int(slot)] += 1
    return vec


def vector_width(slots):
    return max(MIN_SLOTS, (max(slots) + 1) if slots else 0)


class FenceError(Exception):
    pass


# ---------------------------------------------------------------------------
# transports
# ---------------------------------------------------------------------------
class StoreTransport(object):
    """All-reduce through a Redis list (every rank sums every vector)."""

    name = 'store'

    def __init__(self, redis, group, timeout=30.0):
        self.redis = redis
        self.group = group
        self.timeout = timeout

    def allreduce(self, epoch, members, rank, vec, previous=None,
                  fresh=False):
        key = STORE_KEY.format(group=self.group, epoch=epoch)
        self.redis.rpush(key, json.dumps([rank, vec]))
        if rank == 0:
            self.redis.expire(key, 120)
        deadline = time.monotonic() + self.timeout
        while True:
            entries = self.redis.lrange(key, 0, -1)
            if len(entries) >= len(members):
                break
            if time.monotonic() > deadline:
                raise FenceError('store fence epoch %d timed out (%d/%d)' % (
                    epoch, len(entries), len(members)))
            time.sleep(0.002)
        total = [0] * len(vec)
        seen = set()
        for entry in entries:
            r, v = json.loads(entry)
            if r in seen:
                continue
            seen.add(r)
            total = [a + b for a, b in zip(total, v)]
        return total, {}

    def close(self):
        pass


class GlooTransport(object):
    """Per-epoch gloo group over a node-local FileStore (CPU test fake)."""

    name = 'gloo'

    def __init__(self, group, timeout=30.0, root=None):
        self.group = group
        self.timeout = timeout
        self.root = root or tempfile.gettempdir()

    def allreduce(self, epoch, members, rank, vec, previous=None,
                  fresh=False):
        import datetime
        import torch
        import torch.distributed as dist
        safe = self.group.replace('/', '_')
        path = os.path.join(self.root, 'kiosk-fence-%s-%d' % (safe, epoch))
        store = dist.FileStore(path, len(members))
        t0 = time.perf_counter()
        pg = dist.ProcessGroupGloo(store, rank, len(members),
                                   datetime.timedelta(seconds=self.timeout))
        init_ms = (time.perf_counter() - t0) * 1e3
        tensor = torch.tensor(vec, dtype=torch.int64)
        t1 = time.perf_counter()
        pg.allreduce([tensor]).wait()
        us = (time.perf_counter() - t1) * 1e6
        del pg
        return tensor.tolist(), {'init_ms': init_ms, 'allreduce_us': us}

    def close(self):
        pass


class RcclTransport(object):
    """RCCL over xGMI via the native module (``_kiosk_hip.Fence``)."""

    name = 'rccl'

    def __init__(self, redis, group, timeout=60.0, native=None):
        if native is None:
            from ..ops import native as native_ops
            native = native_ops.load()
        self.native = native
        self.redis = redis
        self.group = group
        self.timeout = timeout
        self.comm = None          # native Fence object
        self.comm_members = []    # worker ids in comm rank order

    def _fresh(self, epoch, members, rank):
        if self.comm is not None:
            self.comm.destroy()
            self.comm = None
        key = UID_KEY.format(group=self.group, epoch=epoch)
        if rank == 0:
            uid = self.native.fence_unique_id()
            self.redis.set(key, uid.hex(), ex=120)
        else:
            deadline = time.monotonic() + self.timeout
            while True:
                text = self.redis.get(key)
                if text:
                    uid = bytes.fromhex(text)
                    break
                if time.monotonic() > deadline:
                    raise FenceError('no communicator id for epoch %d' % epoch)
                time.sleep(0.001)
        self.comm = self.native.Fence(uid, len(members), rank,
                                      float(self.timeout))
        self.comm_members = list(members)
        return 'init'

    def _shrink(self, members):
        keep = set(members)
        excluded = [i for i, m in enumerate(self.comm_members)
                    if m not in keep]
        self.comm = self.comm.shrink(excluded, float(self.timeout))
        self.comm_members = [m for m in self.comm_members if m in keep]
        return 'shrink'

    def plan(self, members, previous=None, fresh=False):
        """'reuse' | 'shrink' | 'init' for the next epoch.

        Shrink only when this rank's communicator is exactly the manager's
        last fenced set (``previous``) and the new set is an ordered subset
        of it -- every survivor then takes the same branch."""
        members = list(members)
        if fresh or self.comm is None:
            return 'init'
        if previous is not None and list(previous) != self.comm_members:
            return 'init'
        if self.comm_members == members:
            return 'reuse'
        keep = set(members)
        if (keep < set(self.comm_members) and self.native.fence_can_shrink()
                and [m for m in self.comm_members if m in keep] == members):
            return 'shrink'
        return 'init'

    def allreduce(self, epoch, members, rank, vec, previous=None,
                  fresh=False):
        t0 = time.perf_counter()
        mode = self.plan(members, previous, fresh)
        if mode == 'shrink':
            self._shrink(members)
        elif mode == 'init':
            self._fresh(epoch, members, rank)
        init_ms = (time.perf_counter() - t0) * 1e3
        try:
            result, allreduce_us = self.comm.allreduce(list(vec))
        except Exception:
            self.close()   # never reuse a communicator that failed
            raise
        return list(result), {'init_ms': init_ms, 'allreduce_us': allreduce_us,
                              'mode': mode}

    def close(self):
        if self.comm is not None:
            try:
                self.comm.destroy()
            except Exception:  # pylint: disable=broad-except
                pass
            self.comm = None


# ---------------------------------------------------------------------------
# protocol driver (one per worker)
# ---------------------------------------------------------------------------
class FenceAgent(object):
    """Runs fence commands in order on a background thread."""

    def __init__(self, worker_id, slot, transport, channel=None, events=None):
        self.worker_id = worker_id
        self.slot = int(slot)
        self.transport = transport
        self.channel = channel
        self.events = events
        self._queue = queue.Queue()
        self._aborted = set()
        self.completed = []
        # cleared while an epoch is in flight: the serving loop waits on it
        # (bounded, FENCE_YIELD_MS) so communicator init does not queue
        # behind a whole key of back-to-back forward passes
        self.idle = threading.Event()
        self.idle.set()
        self._thread = threading.Thread(target=self._run, name='fence',
                                        daemon=True)
        self._thread.start()

    def submit(self, message):
        if message.get('cmd') == 'fence_abort':
            self._aborted.add(message.get('epoch'))
            return
        self._queue.put(message)

    def run_epoch(self, message):
        epoch = int(message['epoch'])
        members = list(message['members'])
        slots = [int(s) for s in message.get('slots', range(len(members)))]
        rank = members.index(self.worker_id)
        width = vector_width(slots)
        vec = build_vector(epoch, slots[rank], width)
        t0 = time.perf_counter()
        result, info = self.transport.allreduce(
            epoch, members, rank, vec, previous=message.get('previous'),
            fresh=bool(message.get('fresh')))
        wall_ms = (time.perf_counter() - t0) * 1e3
        expected = expected_vector(epoch, slots, width)
        ok = list(result) == expected
        report = {'epoch': epoch, 'ok': ok, 'rank': rank, 'n': len(members),
                  'transport': self.transport.name, 'wall_ms': wall_ms}
        report.update(info)
        if not ok:
            report['detail'] = 'got %s expected %s' % (result, expected)
        return report

    def _run(self):
        while True:
            message = self._queue.get()
            if message is None:
                return
            epoch = message.get('epoch')
            if epoch in self._aborted:
                continue
            self.idle.clear()
            try:
                report = self.run_epoch(message)
            except Exception as err:  # pylint: disable=broad-except
                logger.warning('fence epoch %s failed: %s', epoch, err)
                report = {'epoch': epoch, 'ok': False, 'detail': str(err),
                          'transport': self.transport.name}
            finally:
                self.idle.set()
            self.completed.append(report)
            if self.events is not None:
                self.events.emit('fence_rank', worker=self.worker_id,
                                 **report)
            if report.get('rank', 0) == 0 or not report['ok']:
                if self.channel is not None:
                    self.channel.emit('fenced', **report)

    def abandon(self):
        """The process is about to exit: stop taking epochs and leave the
        communicator (and any collective still in flight) to process exit."""
        self._queue.put(None)

    def close(self, timeout=5.0):
        """Stop the fence thread and release the communicator.  Returns
        ``False`` if the thread is still inside a collective: the
        communicator is then left alone (destroying it under a running
        all-reduce would be a use-after-free in the native layer) and the
        caller must not reuse this process for another worker."""
        self._queue.put(None)
        self._thread.join(timeout=timeout)
        if self._thread.is_alive():
            logger.warning('fence thread still in a collective at close; '
                           'leaving its communicator to process exit')
            return False
        self.transport.close()
        return True


def choose_transport(kind, backend, redis, group, timeout=60.0):
    if kind in ('auto', ''):
        kind = 'rccl' if backend == 'hip' else 'store'
    if kind == 'rccl':
        return RcclTransport(redis, group, timeout)
    if kind == 'gloo':
        return GlooTransport(group, timeout)
    if kind == 'store':
        return StoreTransport(redis, group, timeout)
    raise ValueError('unknown FENCE transport %r' % kind)


def make_agent_factory(config):
    """Factory used by the worker runtime (called after READY)."""

    def factory(runtime):
        backend = 'hip' if runtime.engine is not None and \
            getattr(runtime.engine, 'name', '') == 'hip' else 'cpu'
        group = '%s/%s' % (os.environ.get('RESOURCE_NAMESPACE', 'default'),
                           os.environ.get('RESOURCE_NAME', 'workers'))
        transport = choose_transport(config.fence, backend, runtime.redis,
                                     group)
        return FenceAgent(config.worker_id, config.slot, transport,
                          channel=runtime.channel, events=runtime.events)
    return factory
