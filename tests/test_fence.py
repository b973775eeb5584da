"""Membership fence protocol, multi-process on CPU.

The production transport is RCCL over xGMI (GPU tests); here the same
FenceAgent protocol runs across real processes over the CPU test fakes:
gloo (torch.distributed, world_size 2) and the Redis-store transport."""
import multiprocessing as mp
import os

import pytest

from kiosk_autoscaler_amd.parallel import fence as fence_mod
from kiosk_autoscaler_amd.parallel.fence import (FenceAgent, GlooTransport,
                                                 StoreTransport,
                                                 build_vector,
                                                 expected_vector)


def test_vectors():
    assert build_vector(3, 2, 8) == [3, 0, 0, 1, 0, 0, 0, 0, 0]
    assert expected_vector(3, [0, 2], 8) == [6, 1, 0, 1, 0, 0, 0, 0, 0]
    assert fence_mod.vector_width([0, 1]) == 8
    assert fence_mod.vector_width([12]) == 13
    # the 72-byte payload of SURVEY N4
    assert len(build_vector(1, 0, 8)) * 8 == 72


class _FakeNative(object):
    """Stands in for _kiosk_hip to exercise RcclTransport planning."""

    def __init__(self):
        self.inits = 0
        self.shrinks = []

    def fence_can_shrink(self):
        return True

    def fence_unique_id(self):
        return b'\x01' * 128

    def Fence(self, uid, n, rank, timeout):
        native = self

        class Comm(object):
            def allreduce(self, vec):
                return list(vec), 1.0

            def shrink(self, excluded, timeout):
                native.shrinks.append(list(excluded))
                return self

            def destroy(self):
                pass
        self.inits += 1
        return Comm()


def test_rccl_transport_plans(redis_client):
    native = _FakeNative()
    t = fence_mod.RcclTransport(redis_client, 'g', native=native)
    a, b, c = 'w-g0-0', 'w-g1-1', 'w-g2-2'
    assert t.plan([a, b]) == 'init'
    t.allreduce(1, [a, b], 0, [1])
    assert redis_client.get(fence_mod.UID_KEY.format(group='g', epoch=1))
    assert t.plan([a, b], previous=[a, b]) == 'reuse'
    assert t.plan([a], previous=[a, b]) == 'shrink'
    assert t.plan([a, c], previous=[a, b]) == 'init'      # grow -> re-init
    assert t.plan([a], previous=[a, c]) == 'init'         # stale view
    assert t.plan([a], previous=[a, b], fresh=True) == 'init'
    _, info = t.allreduce(2, [a], 0, [1], previous=[a, b])
    assert info['mode'] == 'shrink' and native.shrinks == [[1]]
    assert t.comm_members == [a]


def test_store_transport_single_process(redis_client):
    agent = FenceAgent('w0', 0, StoreTransport(redis_client, 'g'))
    try:
        report = agent.run_epoch({'epoch': 4, 'members': ['w0'],
                                  'slots': [0]})
        assert report['ok'] and report['n'] == 1
    finally:
        agent.close()


def _gloo_rank(rank, members, slots, root, out):
    transport = GlooTransport('test/ns', timeout=60, root=root)
    agent = FenceAgent(members[rank], slots[rank], transport)
    try:
        reports = [agent.run_epoch({'epoch': e, 'members': members,
                                    'slots': slots}) for e in (1, 2)]
        out.put((rank, reports))
    finally:
        agent.close()


def _store_rank(rank, members, slots, port, out):
    from kiosk_autoscaler_amd.redisq import StrictRedis
    redis = StrictRedis(host='127.0.0.1', port=port, decode_responses=True)
    agent = FenceAgent(members[rank], slots[rank],
                       StoreTransport(redis, 'ns/w', timeout=30))
    try:
        out.put((rank, agent.run_epoch({'epoch': 7, 'members': members,
                                        'slots': slots})))
    finally:
        agent.close()


def _run_ranks(target, args_for, n):
    ctx = mp.get_context('spawn')
    out = ctx.Queue()
    procs = [ctx.Process(target=target, args=args_for(r) + (out,))
             for r in range(n)]
    for p in procs:
        p.start()
    results = dict(out.get(timeout=120) for _ in range(n))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    return results


@pytest.mark.slow
def test_gloo_fence_world_size_two(tmp_path):
    pytest.importorskip('torch')
    members, slots = ['w-g0-0', 'w-g3-1'], [0, 3]
    results = _run_ranks(_gloo_rank,
                         lambda r: (r, members, slots, str(tmp_path)), 2)
    for rank in (0, 1):
        reports = results[rank]
        assert [r['ok'] for r in reports] == [True, True]
        assert reports[0]['transport'] == 'gloo'
        assert reports[0]['rank'] == rank and reports[0]['n'] == 2


@pytest.mark.slow
def test_store_fence_three_processes(resp_server):
    members, slots = ['a', 'b', 'c'], [0, 1, 5]
    results = _run_ranks(_store_rank,
                         lambda r: (r, members, slots, resp_server.port), 3)
    assert all(results[r]['ok'] for r in range(3))


def test_mismatched_membership_fails(redis_client):
    """A rank that believes in a different set must not report success."""
    transport = StoreTransport(redis_client, 'g', timeout=0.2)
    agent = FenceAgent('x', 0, transport)
    try:
        with pytest.raises(fence_mod.FenceError):
            agent.run_epoch({'epoch': 9, 'members': ['x', 'y'],
                             'slots': [0, 1]})
    finally:
        agent.close()


def test_choose_transport(redis_client):
    assert isinstance(fence_mod.choose_transport('auto', 'cpu', redis_client,
                                                 'g'), StoreTransport)
    assert isinstance(fence_mod.choose_transport('gloo', 'cpu', redis_client,
                                                 'g'), GlooTransport)
    with pytest.raises(ValueError):
        fence_mod.choose_transport('mpi', 'cpu', redis_client, 'g')
    assert os.environ is not None


def test_agent_close_never_destroys_a_busy_communicator():
    """close() while the fence thread is stuck in a collective must leave
    the transport alone and report it (the worker then is not recycled)."""
    import threading
    from kiosk_autoscaler_amd.parallel.fence import FenceAgent
    release = threading.Event()
    closed = []

    class Stuck(object):
        name = 'stuck'

        def allreduce(self, epoch, members, rank, vec, previous=None,
                      fresh=False):
            release.wait(10)
            return vec, {}

        def close(self):
            closed.append(True)

    agent = FenceAgent('w-0', 0, Stuck())
    agent.submit({'cmd': 'fence', 'epoch': 1, 'members': ['w-0'],
                  'slots': [0]})
    import time
    time.sleep(0.1)
    assert agent.close(timeout=0.2) is False and closed == []
    release.set()
    agent._thread.join(5)
