"""Numerics of the gfx950 kernels against plain PyTorch fp32 references.

Runs on an MI355X only (``-m gpu``); every kernel call goes through the
native extension (there is no PyTorch fallback to pass silently)."""
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def mod():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from kiosk_autoscaler_amd.ops import native
    return native.load()


def rand_bf16(*shape, scale=1.0, seed=0):
    g = torch.Generator(device='cuda').manual_seed(seed)
    return ((torch.rand(*shape, generator=g, device='cuda') * 2 - 1)
            * scale).to(torch.bfloat16)


def gelu_tanh(x):
    return 0.5 * x * (1 + torch.tanh(0.7978845608028654 *
                                     (x + 0.044715 * x ** 3)))


@pytest.mark.parametrize('M,N,K', [(128, 128, 64), (256, 384, 512),
                                   (100, 256, 192), (1, 128, 64),
                                   (2048, 1024, 4096)])
def test_gemm_plain(mod, M, N, K):
    from kiosk_autoscaler_amd.ops import kernels
    a = rand_bf16(M, K, seed=1)
    b = rand_bf16(N, K, seed=2)
    c = kernels.gemm(a, b)
    ref = a.float() @ b.float().t()
    err = (c.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item() + 1e-2, err


def test_gemm_identity_asymmetric(mod):
    """A = I with an asymmetric B catches a transposed C-write exactly."""
    from kiosk_autoscaler_amd.ops import kernels
    M = K = 256
    N = 384
    a = torch.eye(M, K, device='cuda', dtype=torch.bfloat16)
    b = (torch.arange(N * K, device='cuda', dtype=torch.float32)
         .reshape(N, K) % 251 - 125).to(torch.bfloat16)
    c = kernels.gemm(a, b)
    assert torch.equal(c, b.t().contiguous()[:M])


def test_gemm_bias_gelu(mod):
    from kiosk_autoscaler_amd.ops import kernels
    M, N, K = 192, 512, 256
    a, b = rand_bf16(M, K, seed=3), rand_bf16(N, K, scale=0.1, seed=4)
    bias = torch.randn(N, device='cuda')
    c = kernels.gemm(a, b, bias=bias, epilogue='gelu')
    ref = gelu_tanh(a.float() @ b.float().t() + bias)
    torch.testing.assert_close(c.float(), ref, atol=2e-2, rtol=2e-2)


def test_gemm_bias_residual(mod):
    from kiosk_autoscaler_amd.ops import kernels
    M, N, K = 130, 256, 512
    a, b = rand_bf16(M, K, seed=5), rand_bf16(N, K, scale=0.05, seed=6)
    bias = torch.randn(N, device='cuda')
    res = rand_bf16(M, N, seed=7)
    c = kernels.gemm(a, b, bias=bias, residual=res, epilogue='residual')
    ref = a.float() @ b.float().t() + bias + res.float()
    torch.testing.assert_close(c.float(), ref, atol=3e-2, rtol=2e-2)


def test_gemm_rejects_bad_shapes(mod):
    from kiosk_autoscaler_amd.ops import kernels
    with pytest.raises(ValueError):
        kernels.gemm(rand_bf16(64, 64), rand_bf16(100, 64))


def test_init_uniform_and_checksum(mod):
    from kiosk_autoscaler_amd.ops import kernels
    t = torch.empty(1 << 20, device='cuda', dtype=torch.bfloat16)
    kernels.init_uniform_(t, 42, -0.5, 0.5)
    f = t.float()
    assert f.min().item() >= -0.5 and f.max().item() <= 0.5
    assert abs(f.mean().item()) < 5e-3
    assert abs(f.std().item() - 1 / (12 ** 0.5)) < 5e-3
    u = torch.empty_like(t)
    kernels.init_uniform_(u, 42, -0.5, 0.5)
    assert torch.equal(t, u)                        # reproducible
    kernels.init_uniform_(u, 43, -0.5, 0.5)
    assert not torch.equal(t, u)
    assert abs(kernels.checksum(t) - f.double().sum().item()) < 1e-2
    odd = torch.empty(1001, device='cuda', dtype=torch.bfloat16)
    kernels.init_uniform_(odd, 1)
    assert abs(kernels.checksum(odd) - odd.double().sum().item()) < 1e-3


def test_engine_matches_reference(mod):
    from kiosk_autoscaler_amd.ops import kernels
    dim, hidden, layers, rows = 256, 1024, 3, 200
    engine = mod.Engine(0, dim, hidden, layers, 256, 5)
    try:
        out = engine.forward(rows, 1, 99)
        ref = kernels.reference_forward_checksum(dim, hidden, layers, rows, 5,
                                                 99)
        assert abs(out['checksum'] - ref) <= 1e-2 * max(1.0, abs(ref)), \
            (out, ref)
        again = engine.forward(rows, 2, 99)        # graph replay, same input
        assert again['graph'] and again['passes'] == 2
        assert abs(again['checksum'] - out['checksum']) < 1e-6
        other = engine.forward(rows, 1, 100)
        assert other['checksum'] != out['checksum']
        stages = engine.stage_times()
        assert list(stages)[:2] == ['engine_enter', 'hip_context']
    finally:
        engine.close()


@pytest.mark.parametrize('dim,hidden,layers,rows', [
    (4096, 16384, 4, 2048),     # the production worker shape (split-K)
    (4096, 16384, 3, 1000),     # odd layer count, ragged rows
    (1024, 4096, 2, 512)])
def test_engine_forward_elementwise(mod, dim, hidden, layers, rows):
    """The whole production forward (graph replay, auto GEMM dispatch with
    the split-K down-projection) elementwise against the fp32 reference --
    a layout or permutation error cannot hide behind a checksum."""
    from kiosk_autoscaler_amd.ops import kernels
    engine = mod.Engine(0, dim, hidden, layers, max(rows, 256), 21)
    try:
        out, ref, stats = kernels.compare_engine_forward(engine, rows, 21, 5)
    finally:
        engine.close()
    assert stats['graph']
    torch.testing.assert_close(out, ref, rtol=3e-2, atol=3e-2)
    assert stats['mean_abs_err'] < 2e-2 * stats['ref_mean_abs']
    # rows are not permuted: each output row is closest to its own
    # reference row
    d = torch.cdist(out[:64], ref[:64])
    assert torch.equal(d.argmin(dim=1), torch.arange(64, device=d.device))


def test_warmstart_touches_every_cu(mod):
    engine = mod.Engine(0, 256, 512, 1, 64, 1)
    try:
        info = engine.warmstart(512)
        cus = torch.cuda.get_device_properties(0).multi_processor_count
        assert info['blocks'] == cus
        assert info['cus_touched'] == cus, info['cus_touched']
        assert info['xccs_touched'] == 8
        # the MFMA loop multiplies real (weight-derived) operands
        assert info['checksum'] != 0.0 and info['checksum'] == \
            info['checksum']
        assert info['kernel_us'] > 0 and info['span_us'] > 0
    finally:
        engine.close()


def test_fence_world_size_one(mod):
    uid = mod.fence_unique_id()
    assert len(uid) == 128
    fence = mod.Fence(uid, 1, 0, 30.0)
    try:
        vec = [7, 0, 1, 0, 0, 0, 0, 0, 0]
        out, us = fence.allreduce(vec)
        assert out == vec and us > 0
    finally:
        fence.destroy()


def test_fence_agent_rccl_transport(mod):
    from kiosk_autoscaler_amd.fakes import FakeRedis
    from kiosk_autoscaler_amd.parallel import FenceAgent, RcclTransport
    transport = RcclTransport(FakeRedis(), 'ns/w', timeout=30.0, native=mod)
    agent = FenceAgent('w-g0-0', 0, transport)
    try:
        r1 = agent.run_epoch({'epoch': 1, 'members': ['w-g0-0'],
                              'slots': [0]})
        assert r1['ok'] and r1['mode'] == 'init'
        r2 = agent.run_epoch({'epoch': 2, 'members': ['w-g0-0'],
                              'slots': [0], 'previous': ['w-g0-0']})
        assert r2['ok'] and r2['mode'] == 'reuse'
    finally:
        agent.close()


def test_node_transport_persistent_world_size_one(mod):
    """The persistent node communicator on RCCL: two-phase connect, then
    many 72-B fences on the same communicator (no re-init per epoch)."""
    import time
    from kiosk_autoscaler_amd.parallel import nodefence
    t = nodefence.RcclNodeTransport(timeout=30.0, native=mod)
    uid = t.make_uid(1)
    t0 = time.perf_counter()
    t.connect(1, 0, 1, uid, should_abort=lambda: False)
    init_ms = (time.perf_counter() - t0) * 1e3
    try:
        lat = []
        for epoch in range(1, 201):
            vec = nodefence.node_vector(epoch, 0, [0] if epoch % 2 else [], 8)
            out, info = t.allreduce(epoch, vec)
            assert out == nodefence.node_expected(
                epoch, 1, [0] if epoch % 2 else [], 8)
            lat.append(info['allreduce_us'])
        lat.sort()
        median = lat[len(lat) // 2]
        print('node comm init %.1f ms, 72-B all-reduce median %.1f us'
              % (init_ms, median))
        assert median < 1000.0          # a fence is sub-millisecond
        assert not t.comm.abort_requested
    finally:
        t.close()
    assert t.comm is None


def test_fence_request_abort_then_destroy(mod):
    """request_abort() from another thread, then destroy(): the owner
    aborts instead of finalizing (no use-after-free)."""
    fence = mod.Fence(1, 0, 30.0)
    fence.connect(mod.fence_unique_id())
    out, _ = fence.allreduce([1, 1, 0, 0, 0, 0, 0, 0, 0])
    assert out[0] == 1
    fence.request_abort()
    assert fence.abort_requested
    fence.destroy()
    fence.destroy()                      # idempotent
    with pytest.raises(RuntimeError):
        fence.allreduce([1])


def test_fence_warmup_and_preinit(mod):
    ms = mod.fence_warmup(60.0)
    assert ms > 0
    stages = mod.preinit_device(0)
    names = list(stages)
    assert names[:2] == ['preinit_enter', 'preinit_context'] and \
        names[-1] == 'preinit_done'
    assert {'preinit_prepared', 'preinit_stream'} <= set(names)
    assert list(stages.values()) == sorted(stages.values())


def test_preinit_pays_the_graph_setup(mod):
    """``preinit_device`` ends with the runtime's one-time graph set-up
    (``graph_prewarm``, profiles/r5_boot) after the stream, and the call is
    repeatable on its own."""
    stages = mod.preinit_device(0)
    names = list(stages)
    assert names.index('preinit_graph_prewarm') == \
        names.index('preinit_stream') + 1
    assert mod.graph_prewarm(0) >= 0.0


def test_stream_graph_replays_kernels_and_copies(mod):
    """``StreamGraph`` (the PyTorch engine's native capture): a pinned-host
    word copied in, a kernel seeded from it, the result copied out -- one
    launch per replay, a new host word per replay; ``abort`` ends a failed
    capture so the stream is usable again."""
    stream = torch.cuda.Stream()
    s = stream.cuda_stream
    seed_host = torch.zeros(1, dtype=torch.int64).pin_memory()
    seed_dev = torch.zeros(1, dtype=torch.int64, device='cuda')
    buf = torch.empty(4096, dtype=torch.bfloat16, device='cuda')
    out_host = torch.zeros(4096, dtype=torch.bfloat16).pin_memory()
    torch.cuda.synchronize()
    graph = mod.StreamGraph(s)
    assert not graph.ready
    with pytest.raises(RuntimeError):
        graph.launch()
    graph.begin()
    mod.memcpy_async(seed_dev.data_ptr(), seed_host.data_ptr(), 8, s)
    mod.init_uniform_bf16_devseed(buf.data_ptr(), buf.numel(),
                                  seed_dev.data_ptr(), -1.0, 1.0, s)
    mod.memcpy_async(out_host.data_ptr(), buf.data_ptr(), buf.numel() * 2, s)
    graph.end()
    assert graph.ready and graph.instantiate_us >= 0
    results = []
    for seed in (5, 6, 5):
        stream.synchronize()
        seed_host[0] = seed
        graph.launch()
        stream.synchronize()
        results.append(out_host.clone())
    # the eager kernel with the same seeds
    for seed, got in zip((5, 6, 5), results):
        ref = torch.empty_like(buf)
        seed_dev.fill_(seed)
        torch.cuda.synchronize()
        mod.init_uniform_bf16_devseed(ref.data_ptr(), ref.numel(),
                                      seed_dev.data_ptr(), -1.0, 1.0, 0)
        torch.cuda.synchronize()
        assert torch.equal(got, ref.cpu())
    assert not torch.equal(results[0], results[1])
    assert torch.equal(results[0], results[2])
    # a capture abandoned half-way leaves the stream capturable again
    graph.begin()
    mod.memset_async(buf.data_ptr(), 0, 64, s)
    graph.abort()
    mod.memset_async(buf.data_ptr(), 0, buf.numel() * 2, s)
    stream.synchronize()
    assert int(buf.float().abs().sum()) == 0
    graph.reset()
    assert not graph.ready


def test_preload_modules_stamps(mod):
    """The context standby's code-object preload (no launch) reports its
    stages in order."""
    stages = mod.preload_modules(0)
    assert list(stages) == ['preload_enter', 'preload_context',
                            'preload_done']
    assert stages['preload_enter'] <= stages['preload_context'] <= \
        stages['preload_done']


@pytest.mark.parametrize('M,N,K', [(256, 256, 32), (300, 512, 96),
                                   (2048, 1024, 4096), (1, 256, 64),
                                   (520, 384, 160), (777, 768, 192),
                                   (256, 512, 128)])
@pytest.mark.parametrize('epilogue', ['none', 'gelu', 'residual'])
@pytest.mark.parametrize('variant', ['256', '256x128', '256w4', '256w4p'])
def test_gemm256_ring_kernel(mod, M, N, K, epilogue, variant):
    """The 256x256 / 256x128 LDS-ring kernels against the fp32 reference
    (odd half counts exercise the clamped tail staging); a shape a variant
    cannot tile (N % 256 for the 256-wide ones, K % 64 for the 4-wave one)
    is refused by the front end before any launch."""
    from kiosk_autoscaler_amd.ops import kernels
    a = rand_bf16(M, K, seed=11)
    b = rand_bf16(N, K, scale=0.1, seed=12)
    bias = torch.randn(N, device='cuda')
    res = rand_bf16(M, N, seed=13)
    if (variant in ('256', '256w4', '256w4p') and N % 256) or \
            (variant in ('256w4', '256w4p') and K % 64):
        with pytest.raises(ValueError, match='needs N'):
            kernels.gemm(a, b, bias=bias, residual=res, epilogue=epilogue,
                         variant=variant)
        return
    ref = a.float() @ b.float().t()
    if epilogue != 'none':
        ref = ref + bias
    if epilogue == 'gelu':
        ref = gelu_tanh(ref)
    if epilogue == 'residual':
        ref = ref + res.float()
    c = kernels.gemm(a, b, bias=bias, residual=res, epilogue=epilogue,
                     variant=variant)
    torch.testing.assert_close(c.float(), ref, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize('M,N,K', [(4000, 4608, 192), (2048, 16384, 256),
                                   (8192, 8192, 128)])
@pytest.mark.parametrize('epilogue', ['none', 'gelu', 'residual'])
def test_gemm256_persistent_walks_many_tiles(mod, M, N, K, epilogue):
    """The persistent 4-wave grid (one workgroup per CU) at shapes with more
    tiles than CUs -- 288, 512 and 1024 tiles, a ragged last row of tiles --
    so workgroups run 2-4 tiles and every tile after the first starts on
    loads prefetched under the previous tile's epilogue."""
    from kiosk_autoscaler_amd.ops import kernels
    a = rand_bf16(M, K, seed=21)
    b = rand_bf16(N, K, scale=0.1, seed=22)
    bias = torch.randn(N, device='cuda')
    res = rand_bf16(M, N, seed=23)
    ref = a.float() @ b.float().t()
    if epilogue != 'none':
        ref = ref + bias
    if epilogue == 'gelu':
        ref = gelu_tanh(ref)
    if epilogue == 'residual':
        ref = ref + res.float()
    c = kernels.gemm(a, b, bias=bias, residual=res, epilogue=epilogue,
                     variant='256w4p')
    torch.testing.assert_close(c.float(), ref, atol=3e-2, rtol=2e-2)
    # bit-identical to the non-persistent 4-wave kernel (same tiles, same
    # K order)
    c4 = kernels.gemm(a, b, bias=bias, residual=res, epilogue=epilogue,
                      variant='256w4')
    assert torch.equal(c, c4)


@pytest.mark.parametrize('M,N,K', [(1280, 2304, 512), (2048, 4096, 256)])
def test_gemm256_group_m_only_reorders_tiles(mod, M, N, K):
    """The tile-row group size (gemm_set_group_m) changes which tiles run
    together, never a tile's result: every group size -- including a ragged
    last group (5 tile rows) -- is bit-identical to the default, for the
    one-tile and the persistent 4-wave grids."""
    from kiosk_autoscaler_amd.ops import kernels
    a = rand_bf16(M, K, seed=31)
    b = rand_bf16(N, K, scale=0.1, seed=32)
    bias = torch.randn(N, device='cuda')
    default = mod.gemm_group_m()
    ref = kernels.gemm(a, b, bias=bias, epilogue='gelu', variant='256w4')
    try:
        for gm in (1, 2, 3, 8, 64):
            mod.gemm_set_group_m(gm)
            assert mod.gemm_group_m() == gm
            for variant in ('256w4', '256w4p'):
                c = kernels.gemm(a, b, bias=bias, epilogue='gelu',
                                 variant=variant)
                assert torch.equal(c, ref), (gm, variant)
    finally:
        mod.gemm_set_group_m(default)
    assert mod.gemm_group_m() == default


def test_gemm256_identity(mod):
    from kiosk_autoscaler_amd.ops import kernels
    M = K = 512
    N = 768
    for n in (768, 1024):
        a = torch.eye(M, K, device='cuda', dtype=torch.bfloat16)
        b = (torch.arange(n * K, device='cuda', dtype=torch.float32)
             .reshape(n, K) % 241 - 120).to(torch.bfloat16)
        if n % 256 == 0:
            c = kernels.gemm(a, b, variant='256w4')
            assert torch.equal(c, b.t().contiguous()[:M]), n
    a = torch.eye(M, K, device='cuda', dtype=torch.bfloat16)
    b = (torch.arange(N * K, device='cuda', dtype=torch.float32)
         .reshape(N, K) % 241 - 120).to(torch.bfloat16)
    for variant in ('256', '256x128', '256w4', '256w4p'):
        if variant in ('256w4', '256w4p') and N % 256:
            continue
        c = kernels.gemm(a, b, variant=variant)
        assert torch.equal(c, b.t().contiguous()[:M]), variant
    assert mod.gemm_pick_variant(2048, 16384, 4096) == 5
    assert mod.gemm_pick_variant(2048, 4096, 16384) == 3
    assert mod.gemm_pick_variant(256, 1024, 1024) == 1


def test_spin_kernel_and_roctx(mod):
    engine = mod.Engine(0, 256, 512, 1, 64, 1)
    try:
        ms = engine.spin(50.0)
        assert 45.0 <= ms < 2000.0, ms
        # the engine still serves after a stall
        out = engine.forward(64, 1, 3)
        assert out['gpu_ms'] > 0
    finally:
        engine.close()
    # roctx calls are safe whether or not a profiler is attached
    assert isinstance(mod.roctx_available(), bool)
    mod.roctx_push('kiosk.test')
    mod.roctx_mark('kiosk.test.mark')
    mod.roctx_pop()


@pytest.mark.parametrize('M,N,K', [(2048, 1024, 4096), (512, 512, 16384),
                                   (300, 512, 8192), (777, 1024, 4096)])
@pytest.mark.parametrize('epilogue', ['none', 'gelu', 'residual'])
@pytest.mark.parametrize('fused', [0, 1])
def test_gemm_splitk(mod, M, N, K, epilogue, fused):
    """Split-K 256x256: two 64-deep-aligned slices run the 4-wave kernel,
    combined through fp32 partial planes + the reduce/epilogue kernel
    (mode 0) or in-launch by each tile's last slice (1); more slices use
    the 8-wave kernel + reduce."""
    from kiosk_autoscaler_amd.ops import kernels
    assert mod.gemm_workspace_bytes(M, N, K) > 0
    default = mod.gemm_splitk_fused()
    mod.gemm_set_splitk_fused(fused)
    try:
        _check_splitk(mod, kernels, M, N, K, epilogue)
        _check_splitk(mod, kernels, M, N, K, epilogue)   # counters re-zeroed
    finally:
        mod.gemm_set_splitk_fused(default)


def _check_splitk(mod, kernels, M, N, K, epilogue):
    a = rand_bf16(M, K, seed=21)
    b = rand_bf16(N, K, scale=0.05, seed=22)
    bias = torch.randn(N, device='cuda')
    res = rand_bf16(M, N, seed=23)
    ref = a.float() @ b.float().t()
    if epilogue != 'none':
        ref = ref + bias
    if epilogue == 'gelu':
        ref = gelu_tanh(ref)
    if epilogue == 'residual':
        ref = ref + res.float()
    c = kernels.gemm(a, b, bias=bias, residual=res, epilogue=epilogue,
                     variant='256splitk')
    torch.testing.assert_close(c.float(), ref, atol=3e-2, rtol=2e-2)
    auto = kernels.gemm(a, b, bias=bias, residual=res, epilogue=epilogue)
    assert torch.equal(auto, c)          # auto picks split-K here


@pytest.mark.parametrize('M,N,K', [(256, 256, 64), (300, 512, 192),
                                   (777, 768, 192), (2048, 1024, 4096),
                                   (1, 256, 64)])
@pytest.mark.parametrize('epilogue', ['none', 'gelu', 'residual'])
def test_gemm256_mfma32_kernel(mod, M, N, K, epilogue):
    """gemm_set_mfma32(1): the 4-wave tile on v_mfma_f32_32x32x16_bf16
    (gemm256m32_kernel) against the fp32 reference -- ragged M, one row,
    a single 64-deep step -- and close to the 16x16x32 kernel (same
    products, K summed in 16- instead of 32-deep MFMA steps)."""
    from kiosk_autoscaler_amd.ops import kernels
    a = rand_bf16(M, K, seed=41)
    b = rand_bf16(N, K, scale=0.1, seed=42)
    bias = torch.randn(N, device='cuda')
    res = rand_bf16(M, N, seed=43)
    ref = a.float() @ b.float().t()
    if epilogue != 'none':
        ref = ref + bias
    if epilogue == 'gelu':
        ref = gelu_tanh(ref)
    if epilogue == 'residual':
        ref = ref + res.float()
    c16 = kernels.gemm(a, b, bias=bias, residual=res, epilogue=epilogue,
                       variant='256w4')
    mod.gemm_set_mfma32(1)
    try:
        c32 = kernels.gemm(a, b, bias=bias, residual=res, epilogue=epilogue,
                           variant='256w4')
    finally:
        mod.gemm_set_mfma32(0)
    torch.testing.assert_close(c32.float(), ref, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(c32.float(), c16.float(), atol=2e-2,
                               rtol=1e-2)


@pytest.mark.parametrize('epilogue', ['gelu', 'residual'])
def test_gemm256_mfma32_splitk_and_forward_shapes(mod, epilogue):
    """The worker's two GEMMs on the 32x32x16 kernel: the up-projection
    (2048x16384x4096: 512 tiles, two per CU) and the split-K
    down-projection (2048x4096x16384: fp32 partial planes + the reduce)."""
    from kiosk_autoscaler_amd.ops import kernels
    for M, N, K in ((2048, 16384, 4096), (2048, 4096, 16384)):
        a = rand_bf16(M, K, seed=51)
        b = rand_bf16(N, K, scale=0.02, seed=52)
        bias = torch.randn(N, device='cuda')
        res = rand_bf16(M, N, seed=53)
        ref = a.float() @ b.float().t() + bias
        ref = gelu_tanh(ref) if epilogue == 'gelu' else ref + res.float()
        mod.gemm_set_mfma32(1)
        try:
            c = kernels.gemm(a, b, bias=bias, residual=res,
                             epilogue=epilogue)
        finally:
            mod.gemm_set_mfma32(0)
        torch.testing.assert_close(c.float(), ref, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize('M,N,K', [(256, 256, 64), (300, 512, 192),
                                   (777, 768, 192), (2048, 1024, 4096),
                                   (1, 256, 64)])
@pytest.mark.parametrize('epilogue', ['none', 'gelu', 'residual'])
def test_gemm256_pair_kernel(mod, M, N, K, epilogue):
    """gemm_set_pair(1): the 256x256 tile on 8 waves, two per SIMD
    (gemm256p_kernel, 128x64 AGPR tiles) against the fp32 reference --
    ragged M, one row, a single 64-deep step -- and bit-identical to the
    4-wave kernel (same MFMAs in the same K order per output)."""
    from kiosk_autoscaler_amd.ops import kernels
    a = rand_bf16(M, K, seed=61)
    b = rand_bf16(N, K, scale=0.1, seed=62)
    bias = torch.randn(N, device='cuda')
    res = rand_bf16(M, N, seed=63)
    ref = a.float() @ b.float().t()
    if epilogue != 'none':
        ref = ref + bias
    if epilogue == 'gelu':
        ref = gelu_tanh(ref)
    if epilogue == 'residual':
        ref = ref + res.float()
    c4 = kernels.gemm(a, b, bias=bias, residual=res, epilogue=epilogue,
                      variant='256w4')
    mod.gemm_set_pair(1)
    try:
        c8 = kernels.gemm(a, b, bias=bias, residual=res, epilogue=epilogue,
                          variant='256w4')
    finally:
        mod.gemm_set_pair(0)
    torch.testing.assert_close(c8.float(), ref, atol=3e-2, rtol=2e-2)
    assert torch.equal(c8, c4)


@pytest.mark.parametrize('epilogue', ['gelu', 'residual'])
def test_gemm256_pair_splitk_and_forward_shapes(mod, epilogue):
    """The worker's two GEMMs on the two-waves-per-SIMD kernel: the
    up-projection (512 tiles) and the split-K down-projection (fp32 partial
    planes + the reduce), elementwise against fp32."""
    from kiosk_autoscaler_amd.ops import kernels
    for M, N, K in ((2048, 16384, 4096), (2048, 4096, 16384)):
        a = rand_bf16(M, K, seed=71)
        b = rand_bf16(N, K, scale=0.02, seed=72)
        bias = torch.randn(N, device='cuda')
        res = rand_bf16(M, N, seed=73)
        ref = a.float() @ b.float().t() + bias
        ref = gelu_tanh(ref) if epilogue == 'gelu' else ref + res.float()
        mod.gemm_set_pair(1)
        try:
            c = kernels.gemm(a, b, bias=bias, residual=res,
                             epilogue=epilogue)
        finally:
            mod.gemm_set_pair(0)
        torch.testing.assert_close(c.float(), ref, atol=3e-2, rtol=2e-2)


def test_splitk_dispatch(mod):
    assert mod.gemm_pick_variant(2048, 4096, 16384, True) == 4
    assert mod.gemm_pick_variant(2048, 4096, 16384, False) == 3
    assert mod.gemm_pick_variant(2048, 16384, 4096, True) == 5
    assert mod.gemm_workspace_bytes(2048, 16384, 4096) == 0
    # two fp32 partial planes + one ticket counter per 256x256 tile
    assert mod.gemm_workspace_bytes(2048, 4096, 16384) == \
        2 * 2048 * 4096 * 4 + 512


def test_engine_cache_across_assignments(mod):
    """A recycled worker keeps its engine (weights, captured graph, pass
    time): the next assignment with the same model reuses it and re-runs
    only the warm-start kernel; a different model frees it first."""
    import time
    from kiosk_autoscaler_amd.worker import main as wmain
    from kiosk_autoscaler_amd.worker.runtime import WorkerConfig
    env = {'MODEL_DIM': '1024', 'MODEL_HIDDEN': '4096', 'MODEL_LAYERS': '2',
           'ROWS_PER_KEY': '256'}
    cfg = WorkerConfig(env, {'worker_id': 'w-g0-a-1'})
    wmain._ENGINES.clear()
    first = wmain._cached_engine('hip', cfg, None)
    try:
        info = first.warmstart()
        assert info['reused'] is False
        wmain._release_engine(first)               # kept, not closed
        assert first.engine is not None
        t0 = time.perf_counter()
        again = wmain._cached_engine('hip', WorkerConfig(
            env, {'worker_id': 'w-g0-a-2'}), None)
        info = again.warmstart()
        reuse_ms = (time.perf_counter() - t0) * 1e3
        assert again is first and info['reused'] is True
        assert info['cus_touched'] > 0 and reuse_ms < 50.0
        out = again.forward(256, 1, 3)
        assert out['gpu_ms'] > 0
        other = wmain._cached_engine('hip', WorkerConfig(
            dict(env, MODEL_LAYERS='1'), {'worker_id': 'w-g0-a-3'}), None)
        assert other is not first and first.engine is None   # evicted
        wmain._release_engine(other)
    finally:
        for eng in list(wmain._ENGINES.values()):
            eng.close()
        wmain._ENGINES.clear()


_EMBRYO_CHILD = r'''
import json, os, sys
from kiosk_autoscaler_amd.ops import native
from kiosk_autoscaler_amd.worker import zygote
mod = native.load()
pre = zygote._HsaPreinit()
pre.DELAY_S = 0.0
request_env = dict(os.environ)
pre.start('0')                      # bound to GPU 0: ROCR_VISIBLE_DEVICES=0
pre.thread.join()
inited = pre.lib is not None
if sys.argv[1] == 'shut':
    # the worker's ROCr settings differ from the init's: shut down
    request_env['HSA_KIOSK_TEST_SETTING'] = 'another'
stamp = pre.settle({'argv': ['--pin', '{"gpu": 0}'], 'env': request_env})
for fd in range(3, 1024):               # as zygote._child does
    if fd not in pre.fds:
        try:
            os.close(fd)
        except OSError:
            pass
stages = dict(mod.preinit_device(0))
print(json.dumps({'inited': inited, 'stamp': stamp,
                  'context_ms': (stages['preinit_context'] -
                                 stages['preinit_enter']) / 1e6,
                  'launched': 'preinit_first_launch' in stages}))
sys.stdout.flush()
os._exit(0)
'''


@pytest.mark.parametrize('mode', ['keep', 'shut'])
def test_embryo_rocr_preinit_then_device(mode):
    """An embryo's early ROCr init (worker/zygote.py ``_HsaPreinit``): ROCr
    initialised before HIP, kept (same pin) or shut down and initialised
    again by HIP (another pin), leaves a process whose device opens and
    runs its first kernel.  Fresh processes: the init is once per process."""
    import json
    import os
    import subprocess
    import sys
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root)
    out = subprocess.run([sys.executable, '-c', _EMBRYO_CHILD, mode],
                         capture_output=True, text=True, timeout=90,
                         env=env, cwd=root)
    assert out.returncode == 0, out.stderr[-2000:]
    row = json.loads(out.stdout.strip().splitlines()[-1])
    assert row['inited'] and row['launched']
    assert (row['stamp'] is not None) == (mode == 'keep')
