"""The PyTorch-ROCm worker engine on the hand-written kernels
(models/torch_kiosk.py, VERDICT r3 missing 2 / next-step 3): full-output
numerics against the fp32 PyTorch reference, bit-equality with the
built-in native engine, one-graph-launch warm start and forward, and the
engine serving keys through a real worker process on MI355X."""
import json
import os
import subprocess
import sys
import time

import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

SPEC = 'kiosk_autoscaler_amd.models.torch_kiosk:TorchKioskEngine'


@pytest.fixture(scope='module')
def cuda():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from kiosk_autoscaler_amd.ops import native
    native.load()       # torch first: one HIP runtime
    return torch.device('cuda')


def _cfg(dim, hidden, layers, rows, seed=21):
    from kiosk_autoscaler_amd.worker.runtime import WorkerConfig
    env = {'MODEL_DIM': str(dim), 'MODEL_HIDDEN': str(hidden),
           'MODEL_LAYERS': str(layers), 'ROWS_PER_KEY': str(rows),
           'MODEL_SEED': str(seed)}
    return WorkerConfig(env, {'worker_id': 'w'})


@pytest.mark.parametrize('dim,hidden,layers,rows', [
    (1024, 4096, 2, 512),
    (4096, 16384, 4, 2048),      # the benchmark model: split-K down-proj
])
def test_full_output_matches_fp32_reference(cuda, dim, hidden, layers, rows):
    from kiosk_autoscaler_amd.models.torch_kiosk import TorchKioskEngine
    from kiosk_autoscaler_amd.ops import kernels
    engine = TorchKioskEngine(_cfg(dim, hidden, layers, rows))
    try:
        out = engine.output(rows, 5).float()
        weights = kernels.model_weights(dim, hidden, layers, 21)
        x = torch.empty((rows, dim), dtype=torch.bfloat16, device='cuda')
        kernels.init_uniform_(x, 5, -1.0, 1.0)
        ref = kernels.reference_forward(x, weights).float()
        torch.testing.assert_close(out, ref, rtol=3e-2, atol=3e-2)
        assert (out - ref).abs().mean() < 2e-2 * ref.abs().mean()
        d = torch.cdist(out[:64], ref[:64])
        assert torch.equal(d.argmin(dim=1),
                           torch.arange(64, device=d.device))
        # a different seed is a different input, through the same graph
        other = engine.output(rows, 6).float()
        assert not torch.equal(other, out)
        assert len(engine.graphs) == 1
    finally:
        engine.close()


def test_bit_identical_to_the_native_engine(cuda):
    """Same kernels, same seeds, same variant choices: the PyTorch engine
    and the built-in one serve the same bytes."""
    from kiosk_autoscaler_amd.models.torch_kiosk import TorchKioskEngine
    from kiosk_autoscaler_amd.ops import kernels, native
    mod = native.load()
    dim, hidden, layers, rows = 1024, 4096, 2, 512
    engine = TorchKioskEngine(_cfg(dim, hidden, layers, rows))
    native_engine = mod.Engine(0, dim, hidden, layers, rows, 21)
    try:
        ours = engine.output(rows, 9)
        result = native_engine.forward(rows, 1, 9)
        theirs = kernels.engine_output(native_engine, rows)
        assert torch.equal(ours, theirs)
        # the key's checksum: the same partials summed in the same order,
        # without a torch kernel on the serving path
        assert engine.checksum() == result['checksum']
        served = engine.infer([{'rows': rows, 'seed': 9, 'service_ms': 0}])
        assert served[0]['output_sum'] == '%.6e' % result['checksum']
    finally:
        native_engine.close()
        engine.close()


def test_warmstart_and_forward_are_graph_launches(cuda):
    from kiosk_autoscaler_amd.models.torch_kiosk import TorchKioskEngine
    engine = TorchKioskEngine(_cfg(1024, 4096, 2, 512))
    try:
        info = engine.warmstart()
        cus = torch.cuda.get_device_properties(0).multi_processor_count
        assert info['graph'] and info['blocks'] == cus
        rec = engine.warm_record.view(-1, 8).cpu()
        # every block wrote its hardware ids and a non-zero MFMA sum
        assert int((rec[:, 6] != 0).sum()) == cus
        # after warm-up a READY costs one graph launch: well under 5 ms
        t0 = time.perf_counter()
        engine.warmstart()
        assert time.perf_counter() - t0 < 0.005
        outs = engine.infer([{'rows': 512, 'seed': 3, 'service_ms': 0}])
        assert outs[0]['passes'] == 1 and outs[0]['engine'] == 'torch-kiosk'
    finally:
        engine.close()


def test_engine_reuses_the_preinit_stream_and_a_dlpack_arena(cuda):
    """Standby boot path: the engine wraps the stream preinit_device warmed
    (no new hardware queue) and hands it back on close; its arena is one
    hipMalloc handed over by DLPack and freed with the engine."""
    from kiosk_autoscaler_amd.models.torch_kiosk import TorchKioskEngine
    from kiosk_autoscaler_amd.ops import native
    mod = native.load()
    mod.preinit_device(0)
    free0 = mod.mem_info()[0]
    stages = {}
    engine = TorchKioskEngine(_cfg(1024, 4096, 2, 512),
                              lambda name: stages.setdefault(name, 1))
    handle = engine._stream_handle
    try:
        assert handle and engine.stream.cuda_stream == handle
        assert {'stream_ready', 'arena_allocated', 'graphs_ready'} <= set(
            stages)
        assert engine.hbm_bytes() == engine.arena.numel()
        assert free0 - mod.mem_info()[0] >= engine.hbm_bytes()
        engine.warmstart()
        out = engine.infer([{'rows': 512, 'seed': 4, 'service_ms': 0}])
        assert out[0]['passes'] == 1
    finally:
        engine.close()
    engine.close()                       # idempotent
    torch.cuda.synchronize()
    # the arena is freed (up to the allocator's rounding) ...
    assert mod.mem_info()[0] > free0 - (64 << 20)
    # ... and the stream is kept again for the next engine
    again = mod.take_stream(0)
    assert again == handle
    mod.return_stream(again, 0)


_COMGR_CHILD = r'''
import json, sys
sys.path.insert(0, sys.argv[1])
from kiosk_autoscaler_amd.ops import native, kernels
mod = native.load(torch_first=True)        # the worker's load order
import torch
from kiosk_autoscaler_amd.models.torch_kiosk import TorchKioskEngine
from kiosk_autoscaler_amd.worker.runtime import WorkerConfig
stages = dict(mod.preinit_device(0))
cfg = WorkerConfig({'MODEL_DIM': '1024', 'MODEL_HIDDEN': '4096',
                    'MODEL_LAYERS': '2', 'ROWS_PER_KEY': '512',
                    'MODEL_SEED': '21'}, {'worker_id': 'w'})
engine = TorchKioskEngine(cfg)
ours = engine.output(512, 9)
ref_engine = mod.Engine(0, 1024, 4096, 2, 512, 21)
ref_engine.forward(512, 1, 9)
same = bool(torch.equal(ours, kernels.engine_output(ref_engine, 512)))
# torch's own blit kernels and BLAS after the comgr swap
a = torch.full((256, 256), 0.25, device='cuda', dtype=torch.bfloat16)
blas = float((a @ a).float().sum().cpu())
ref_engine.close()
engine.close()
maps = [l.split()[-1] for l in open('/proc/self/maps')]
print(json.dumps({
    'same': same, 'blas': blas,
    'stream_ms': (stages['preinit_stream'] - stages['preinit_prepared']) / 1e6,
    'comgr': sorted({m for m in maps if 'comgr' in m}),
    'hip': sorted({m for m in maps if 'libamdhip64' in m})}))
'''


def test_worker_load_order_runs_rocm_comgr_under_torch(cuda):
    """``native.load(torch_first=True)`` (the PyTorch worker's load order)
    maps ROCm's comgr under torch's own HIP runtime: the engine still
    serves the built-in engine's bytes, torch's blit kernels and BLAS still
    work, and the first stream no longer pays torch's uncached blit-kernel
    front end (profiles/r4_stream)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, '-c', _COMGR_CHILD, root],
                         stdout=subprocess.PIPE, timeout=120, check=True)
    row = json.loads(out.stdout.decode().strip().splitlines()[-1])
    print(row)
    assert row['same'] and row['blas'] == 256 * 256 * 256 * 0.0625
    assert len(row['comgr']) == 1 and row['comgr'][0].startswith('/opt/rocm')
    assert len(row['hip']) == 1 and 'torch' in row['hip'][0]


def test_torch_worker_serves_keys_through_the_manager(resp_server):
    """A real PyTorch-ROCm worker process (zygote-forked, torch imported,
    native kernels on torch's allocator and stream) scales up, serves keys
    with the engine and reports the graph warm start."""
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from kiosk_autoscaler_amd import gpumgr
    from kiosk_autoscaler_amd.config import Config, Settings
    from kiosk_autoscaler_amd.redisq import StrictRedis
    from kiosk_autoscaler_amd.utils.events import EventLog
    env = {'REDIS_HOST': resp_server.host, 'REDIS_PORT': str(resp_server.port),
           'QUEUES': 'predict', 'RESOURCE_NAME': 'tk', 'MAX_PODS': '1',
           'WORKER_BACKEND': 'hip', 'WARM_POOL': '1', 'FENCE': 'auto',
           'REDIS_INTERVAL': '0', 'GPU_IDS': '0', 'MODEL': '1024x4096x2',
           'ROWS_PER_KEY': '512',
           'POOL_IDLE_RELEASE_S': '0'}
    s = Settings(Config(environ=env, use_files=False))
    client = StrictRedis(host=resp_server.host, port=resp_server.port,
                         decode_responses=True)
    events = EventLog(source='test')
    events.keep = True
    manager = gpumgr.build_manager(s, redis_client=client, events=events,
                                   extra_env={'WORKER_ENGINE': SPEC}).start()
    try:
        deadline = time.monotonic() + 120
        while not (manager.standbys and all(
                p.booted for p in manager.standbys.values())):
            assert time.monotonic() < deadline
            time.sleep(0.05)
        for i in range(3):
            client.hset('predict:t%d' % i, mapping={'status': 'new',
                                                    'rows': 512, 'seed': i})
            client.lpush('predict', 'predict:t%d' % i)
        manager.patch_namespaced_deployment('tk', 'default',
                                            {'spec': {'replicas': 1}})
        deadline = time.monotonic() + 60
        while not all(client.hget('predict:t%d' % i, 'status') == 'done'
                      for i in range(3)):
            assert time.monotonic() < deadline
            time.sleep(0.05)
        assert client.hget('predict:t0', 'engine') == 'torch-kiosk'
        ups = [e for e in events.records if e['ev'] == 'worker_up']
        assert ups and ups[0]['ready_s'] < 0.5, ups
        print('torch-kiosk worker: assign -> READY %.1f ms' %
              (1e3 * ups[0]['ready_s']))
    finally:
        manager.patch_namespaced_deployment('tk', 'default',
                                            {'spec': {'replicas': 0}})
        manager.stop(timeout=30)
    assert os.environ.get('WORKER_ENGINE') is None
