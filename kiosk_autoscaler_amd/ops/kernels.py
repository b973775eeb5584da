"""torch-tensor front end for the native gfx950 kernels.

Every function here launches a hand-written HIP kernel from ``_kiosk_hip``
on the current PyTorch stream; none falls back to a PyTorch op.  The
``reference_*`` helpers are the plain fp32 PyTorch references the numerics
tests compare against.
"""
import math

from . import native

EPILOGUES = {'none': 0, 'gelu': 1, 'bias_gelu': 1, 'residual': 2,
             'bias_residual': 2}


def _stream():
    import torch
    return torch.cuda.current_stream().cuda_stream


def _check_bf16(t, name):
    import torch
    if t.dtype != torch.bfloat16 or not t.is_cuda or not t.is_contiguous():
        raise ValueError('%s must be a contiguous bf16 CUDA tensor' % name)


VARIANTS = {'auto': 0, '128': 1, '256': 2, '256x128': 3, '256splitk': 4,
            '256w4': 5, '256w4p': 6}


def gemm(a, b, bias=None, residual=None, epilogue='none', out=None,
         variant='auto'):
    """``epi(a @ b.T)`` with a: [M, K], b: [N, K] (bf16) -> [M, N] bf16.

    ``epilogue``: ``'none'``, ``'gelu'`` (``gelu_tanh(a@b.T + bias)``) or
    ``'residual'`` (``a@b.T + bias + residual``).  ``variant``: ``'auto'``
    (256x256 LDS-ring kernel when the grid fills the chip, else the 256x128
    ring when that does, else 128x128; split-K 256x256 where the grid alone
    would leave CUs idle), ``'128'``, ``'256'``, ``'256x128'`` or
    ``'256splitk'`` (fp32 partials in a temporary workspace + one fused
    reduce/epilogue kernel), ``'256w4'`` (256x256 ring, 4 waves of
    128x128 outputs) or ``'256w4p'`` (the same as a persistent grid: one
    workgroup per CU walks the tiles, the next tile's first loads overlap
    the epilogue)."""
    import torch
    mod = native.load()
    _check_bf16(a, 'a')
    _check_bf16(b, 'b')
    M, K = a.shape
    N, K2 = b.shape
    if K != K2:
        raise ValueError('inner dimensions differ: %d vs %d' % (K, K2))
    if variant == '256splitk':
        if mod.gemm_workspace_bytes(M, N, K) == 0:
            raise ValueError('split-K does not apply to M=%d N=%d K=%d '
                             '(the 256x256 grid already fills the chip, or '
                             'K is too short)' % (M, N, K))
    elif variant in ('256', '256x128', '256w4', '256w4p'):
        bn = 128 if variant == '256x128' else 256
        kq = 64 if variant in ('256w4', '256w4p') else 32
        if M < 1 or N % bn or K % kq or K < kq:
            raise ValueError('the 256x%d kernel needs N %% %d == 0 and '
                             'K %% %d == 0 (M=%d N=%d K=%d)'
                             % (bn, bn, kq, M, N, K))
    elif not mod.gemm_shape_ok(M, N, K):
        raise ValueError('unsupported GEMM shape M=%d N=%d K=%d (need N %% 128'
                         ' == 0, K %% 64 == 0)' % (M, N, K))
    epi = EPILOGUES[epilogue]
    if epi and (bias is None or bias.dtype != torch.float32
                or bias.numel() != N or not bias.is_contiguous()):
        raise ValueError('epilogue %r needs an fp32 bias of %d' % (epilogue, N))
    if epi == 2:
        _check_bf16(residual, 'residual')
        if tuple(residual.shape) != (M, N):
            raise ValueError('residual must be [M, N]')
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    ws_bytes = mod.gemm_workspace_bytes(M, N, K) \
        if variant in ('auto', '256splitk') else 0
    workspace = torch.empty(max(1, ws_bytes // 4), dtype=torch.float32,
                            device=a.device) if ws_bytes else None
    mod.gemm(a.data_ptr(), b.data_ptr(), out.data_ptr(),
             bias.data_ptr() if bias is not None else 0,
             residual.data_ptr() if residual is not None else 0,
             M, N, K, epi, _stream(), VARIANTS[variant],
             workspace.data_ptr() if workspace is not None else 0, ws_bytes)
    return out


def init_uniform_(t, seed, lo=-1.0, hi=1.0):
    """Fill a bf16 or fp32 CUDA tensor with the on-device generator."""
    import torch
    mod = native.load()
    if not t.is_contiguous() or not t.is_cuda:
        raise ValueError('tensor must be contiguous on the GPU')
    if t.dtype == torch.bfloat16:
        mod.init_uniform_bf16(t.data_ptr(), t.numel(), int(seed), lo, hi,
                              _stream())
    elif t.dtype == torch.float32:
        mod.init_uniform_f32(t.data_ptr(), t.numel(), int(seed), lo, hi,
                             _stream())
    else:
        raise ValueError('init_uniform_ supports bf16 / fp32')
    return t


def checksum(t):
    """fp32 sum of a bf16 tensor via the deterministic partial-sum kernel."""
    import torch
    mod = native.load()
    _check_bf16(t, 't')
    partials = torch.empty(mod.sum_blocks, dtype=torch.float32,
                           device=t.device)
    mod.partial_sums(t.data_ptr(), t.numel(), partials.data_ptr(), _stream())
    return float(partials.double().sum().item())


def model_weights(dim, hidden, layers, seed, device='cuda', alloc=None):
    """Regenerate the Engine's weights (same seeds and bounds) as tensors.
    ``alloc(shape, dtype)`` places them (e.g. in one arena); default
    ``torch.empty`` on ``device``."""
    import torch
    if alloc is None:
        def alloc(shape, dtype):
            return torch.empty(shape, dtype=dtype, device=device)
    bd, bh = 1.0 / math.sqrt(dim), 1.0 / math.sqrt(hidden)
    weights = []
    for layer in range(layers):
        s = seed * 1000003 + 16 * layer
        w1 = alloc((hidden, dim), torch.bfloat16)
        b1 = alloc((hidden,), torch.float32)
        w2 = alloc((dim, hidden), torch.bfloat16)
        b2 = alloc((dim,), torch.float32)
        init_uniform_(w1, s + 1, -bd, bd)
        init_uniform_(b1, s + 2, -bd, bd)
        init_uniform_(w2, s + 3, -bh, bh)
        init_uniform_(b2, s + 4, -bh, bh)
        weights.append((w1, b1, w2, b2))
    return weights


def reference_forward(x, weights):
    """fp32 PyTorch reference of the worker model with the kernels' bf16
    storage points (hidden activation and every layer output)."""
    import torch
    from ..models.mlp import torch_reference
    for w1, b1, w2, b2 in weights:
        x = torch_reference(x, w1, b1, w2, b2).to(torch.bfloat16)
    return x


def reference_forward_checksum(dim, hidden, layers, rows, model_seed,
                               input_seed):
    import torch
    weights = model_weights(dim, hidden, layers, model_seed)
    x = torch.empty((rows, dim), dtype=torch.bfloat16, device='cuda')
    init_uniform_(x, input_seed, -1.0, 1.0)
    y = reference_forward(x, weights)
    return float(y.double().sum().item())


def engine_output(engine, rows):
    """The last ``Engine.forward`` output as a ``[rows, dim]`` bf16 tensor."""
    import torch
    out = torch.empty((rows, engine.dim), dtype=torch.bfloat16,
                      device='cuda')
    torch.cuda.synchronize()
    engine.copy_output(out.data_ptr(), rows)
    return out


def compare_engine_forward(engine, rows, model_seed, input_seed):
    """Run one (graph-replayed) ``Engine.forward`` and compare its whole
    output elementwise against :func:`reference_forward` (fp32 PyTorch with
    the kernels' bf16 storage points).  Returns ``(out, ref, stats)``."""
    import torch
    engine.prepare(rows)                 # capture: the forward is a replay
    result = engine.forward(rows, 1, input_seed)
    out = engine_output(engine, rows).float()
    weights = model_weights(engine.dim, engine.hidden, engine.layers,
                            model_seed)
    x = torch.empty((rows, engine.dim), dtype=torch.bfloat16, device='cuda')
    init_uniform_(x, input_seed, -1.0, 1.0)
    ref = reference_forward(x, weights).float()
    err = (out - ref).abs()
    stats = {'max_abs_err': float(err.max()),
             'mean_abs_err': float(err.mean()),
             'ref_mean_abs': float(ref.abs().mean()),
             'checksum': result['checksum'], 'graph': result['graph'],
             'gpu_ms': result['gpu_ms']}
    return out, ref, stats
