"""Serving loop yields to an in-flight fence epoch (FENCE_YIELD_MS).

RCCL's communicator init waits for the device to go idle; under a key's
back-to-back forward chunks it finished only when the key did (~1 s
instead of ~45 ms idle, profiles/r1_final_check).  The loop pauses while
``FenceAgent.idle`` is clear, bounded, and the pause is not service time
nor GPU-busy time.  CPU-only: the native engine is replaced by a stub that
sleeps its pass time.
"""
import threading
import time

from kiosk_autoscaler_amd.bench import metrics
from kiosk_autoscaler_amd.models import mlp
from kiosk_autoscaler_amd.parallel import fence


class _StubNative(object):
    def __init__(self, pass_ms=1.0):
        self.pass_ms = pass_ms
        self.calls = []

    def forward(self, rows, passes, seed):
        self.calls.append((time.perf_counter(), passes))
        time.sleep(self.pass_ms * passes / 1e3)
        return {'gpu_ms': self.pass_ms * passes, 'checksum': 1.0}


def _engine(pass_ms=1.0):
    eng = mlp.HipMlpEngine.__new__(mlp.HipMlpEngine)
    eng.engine = _StubNative(pass_ms)
    eng.pass_ms = {64: pass_ms}
    return eng


def test_no_pause_when_fence_idle():
    eng = _engine()
    idle = threading.Event()
    idle.set()
    out = eng.forward_for(64, 30.0, 0, chunk_ms=5.0, pause=(idle, 250.0))
    assert out['paused_ms'] == 0.0
    assert out['passes'] >= 20


def test_pause_until_fence_done_and_not_counted_as_service():
    eng = _engine()
    idle = threading.Event()          # a fence epoch is in flight
    threading.Timer(0.06, idle.set).start()
    t0 = time.perf_counter()
    out = eng.forward_for(64, 30.0, 0, chunk_ms=5.0, pause=(idle, 250.0))
    wall = (time.perf_counter() - t0) * 1e3
    assert 40.0 <= out['paused_ms'] <= 200.0
    # the pause happened before any chunk was issued
    assert eng.engine.calls[0][0] - t0 >= 0.04
    # full service still delivered after the pause
    assert out['ms'] >= 25.0 and wall >= out['paused_ms'] + 25.0


def test_pause_is_bounded():
    eng = _engine()
    idle = threading.Event()          # never completes
    out = eng.forward_for(64, 20.0, 0, chunk_ms=5.0, pause=(idle, 30.0))
    assert 25.0 <= out['paused_ms'] <= 120.0
    assert out['passes'] >= 10


class _SlowTransport(object):
    name = 'stub'

    def __init__(self, delay):
        self.delay = delay

    def allreduce(self, epoch, members, rank, vec, previous=None,
                  fresh=False):
        time.sleep(self.delay)
        return (fence.expected_vector(epoch, [0], fence.vector_width([0])),
                {'init_ms': self.delay * 1e3})

    def close(self):
        pass


def test_agent_idle_event_brackets_epoch():
    agent = fence.FenceAgent('w0', 0, _SlowTransport(0.05))
    assert agent.idle.is_set()
    agent.submit({'cmd': 'fence', 'epoch': 1, 'members': ['w0'],
                  'slots': [0]})
    deadline = time.monotonic() + 2.0
    while agent.idle.is_set() and not agent.completed:
        assert time.monotonic() < deadline
        time.sleep(0.001)
    assert agent.idle.wait(2.0)
    assert agent.completed and agent.completed[0]['ok']
    assert agent.close()


def test_paused_time_is_not_gpu_busy():
    ms = 1000000
    events = [
        {'ev': 'worker_assigned', 'worker': 'w', 't': 0},
        {'ev': 'key_start', 'worker': 'w', 'item': 'k', 't': 0},
        {'ev': 'key_done', 'worker': 'w', 'item': 'k', 't': 1000 * ms,
         'paused_ms': 100.0},
        {'ev': 'worker_exit', 'worker': 'w', 't': 2000 * ms},
    ]
    idle, alive_s, busy_s = metrics.gpu_idle(events, 0, 2000 * ms)
    assert abs(busy_s - 0.9) < 1e-9 and abs(alive_s - 2.0) < 1e-9
    assert abs(idle - 55.0) < 1e-9


def test_channel_routes_fence_commands_off_the_main_thread():
    import json
    import os
    from kiosk_autoscaler_amd.worker.channel import Channel
    r, w = os.pipe()
    chan = Channel(cmd_fd=r)
    got = []
    arrived = threading.Event()

    def handler(message):
        got.append((message, threading.current_thread().name))
        arrived.set()
    chan.direct['fence'] = handler
    chan.start_reader()
    for msg in ({'cmd': 'drain'}, {'cmd': 'fence', 'epoch': 3}):
        os.write(w, (json.dumps(msg) + '\n').encode())
    assert arrived.wait(2.0)
    assert got[0][0]['epoch'] == 3 and got[0][1] == 'worker-cmd'
    assert chan.commands.get(timeout=2.0)['cmd'] == 'drain'
    assert chan.commands.empty()
    os.close(w)
    assert chan.commands.get(timeout=2.0)['cmd'] == 'eof'
    os.close(r)


def test_short_chunks_while_fence_busy_without_pausing():
    eng = _engine()
    idle = threading.Event()          # fence in flight for ~40 ms
    threading.Timer(0.04, idle.set).start()
    out = eng.forward_for(64, 80.0, 0, chunk_ms=20.0, pause=(idle, 0.0, 2.0))
    assert out['paused_ms'] == 0.0
    sizes = [n for _, n in eng.engine.calls]
    assert sizes[0] <= 2 and max(sizes) >= 10
