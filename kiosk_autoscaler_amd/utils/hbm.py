"""HBM sizing for ``KEYS_PER_POD`` (BASELINE config 5).

A worker keeps its model resident in HBM and, in one-shot ``job`` mode,
batches up to ``KEYS_PER_POD`` keys into one forward pass.  This module
computes how many keys' working sets fit beside the weights on one MI355X
(288 GB HBM3E) and clamps / warns when the configured value does not fit:

    max_kpp = max k such that engine_bytes(rows = k x R) fits
              in HBM - reserve

``engine_bytes`` is the engine's one device arena, byte for byte
(``Engine::Engine``, csrc/runtime/engine.cpp, and the PyTorch engine's
arena, models/torch_kiosk.py): per layer bf16 ``W1 [H,D]``, fp32 ``b1
[H]``, bf16 ``W2 [D,H]``, fp32 ``b2 [D]``; then bf16 ``x``, ``y [rows,D]``
and ``h [rows,H]``, the fp32 partial sums, the seed word and the split-K
workspace (fp32 partial planes for the row counts whose GEMM grid would
leave CUs idle, ``gemm256_splitk_workspace``), every piece 256-B aligned
(the former model counted bf16 biases and no
workspace).  The per-key cost is the arena's growth per ``R`` rows.
"""
import functools
import logging
import os

MI355X_HBM_BYTES = 288 * 10 ** 9   # spec capacity (decimal GB)
BF16 = 2
FP32 = 4
ALIGN = 256
SUM_BLOCKS = 1024                  # kSumBlocks (csrc/kernels/kernels.hpp)
WARM_RECORD_BYTES = 256 * 8 * 4    # the warm-start record (one per CU)

logger = logging.getLogger('HbmSizing')


def _align(n):
    return (n + ALIGN - 1) // ALIGN * ALIGN


def model_bytes(dim, hidden, layers):
    """The weights as the arena holds them (bf16 matrices, fp32 biases)."""
    return layers * (_align(hidden * dim * BF16) + _align(hidden * FP32) +
                     _align(dim * hidden * BF16) + _align(dim * FP32))


def splitk_splits(m, n, k):
    """``gemm256_splits``: split K while the 256x256 grid leaves CUs idle,
    each slice keeps >= 2048 of K, slices stay 32-aligned."""
    tiles = -(-m // 256) * (n // 256)
    if tiles >= 256 or n % 256 or k % 32:
        return 1
    s = 1
    while s < 4 and tiles * s < 256 and k % (2 * s * 32) == 0 and \
            k // (2 * s) >= 2048:
        s *= 2
    return s


def splitk_workspace_bytes(m, n, k):
    """``gemm256_splitk_workspace``: fp32 partial planes + tile counters."""
    s = splitk_splits(m, n, k)
    if s <= 1:
        return 0
    tiles = -(-m // 256) * (n // 256)
    return s * m * n * FP32 + (tiles * 4 + 255) // 256 * 256


def workspace_bytes(max_rows, dim, hidden):
    """The engine's workspace: the largest either GEMM wants for any row
    count up to ``max_rows`` (probed at 256-row steps, as the engine).
    Only row counts whose grid has fewer than 256 tiles split, so the
    probe stops there: a handful of steps whatever ``max_rows`` (this runs
    on the manager's assignment path)."""
    narrow = max(1, min(dim, hidden) // 256)       # tiles per 256 rows
    stop = min(max_rows, 256 * -(-256 // narrow))
    ws = 0
    for m in range(256, stop + 256, 256):
        rows = min(m, max_rows)
        ws = max(ws, splitk_workspace_bytes(rows, hidden, dim),
                 splitk_workspace_bytes(rows, dim, hidden))
    return ws


@functools.lru_cache(maxsize=4096)
def engine_bytes(dim, hidden, layers, max_rows):
    """Device bytes of an engine with room for ``max_rows`` rows (the
    built-in engine's arena plus its warm-start record)."""
    max_rows = max(int(max_rows), 256)
    return (model_bytes(dim, hidden, layers) +
            2 * _align(max_rows * dim * BF16) +
            _align(max_rows * hidden * BF16) + _align(SUM_BLOCKS * FP32) +
            _align(8) + _align(workspace_bytes(max_rows, dim, hidden)) +
            WARM_RECORD_BYTES)


def per_key_bytes(rows, dim, hidden):
    """Activation bytes one more key of ``rows`` rows adds (x, y, h)."""
    return 2 * rows * dim * BF16 + rows * hidden * BF16


def max_keys_per_pod(hbm_bytes, weights, per_key, reserve=8 << 30):
    free = hbm_bytes - reserve - weights
    if per_key <= 0:
        raise ValueError('per_key_bytes must be positive')
    return max(0, free // per_key)


def device_hbm_bytes(pci=None):
    """HBM capacity without touching HIP: sysfs VRAM size, else the spec."""
    paths = []
    if pci:
        paths.append('/sys/bus/pci/devices/%s/mem_info_vram_total' % pci)
    paths.extend('/sys/class/drm/card%d/device/mem_info_vram_total' % i
                 for i in range(16))
    for path in paths:
        try:
            with open(path) as handle:
                value = int(handle.read().strip())
            if value > 0:
                return value
        except (OSError, ValueError):
            continue
    return MI355X_HBM_BYTES


def _fit(budget, dim, hidden, layers, rows, per_key):
    """Largest k >= 0 with engine_bytes(k x rows) <= budget (``per_key``:
    an operator's override of the per-key activation bytes)."""
    if per_key:
        base = engine_bytes(dim, hidden, layers, rows) - per_key_bytes(
            rows, dim, hidden)
        return max(0, (budget - base) // per_key)
    if engine_bytes(dim, hidden, layers, rows) > budget:
        return 0
    # engine_bytes(k x rows) = fixed + k x per_key + workspace(k x rows),
    # the workspace never above its cap: the k that fits with the cap is a
    # lower bound, a few steps below the answer (this runs on the
    # manager's assignment path: a handful of evaluations, not a search)
    per = per_key_bytes(rows, dim, hidden)
    cap = workspace_bytes(1 << 30, dim, hidden)
    fixed = engine_bytes(dim, hidden, layers, rows) - per - \
        _align(workspace_bytes(max(rows, 256), dim, hidden))
    k = max(1, (budget - fixed - _align(cap)) // per)
    while engine_bytes(dim, hidden, layers, (k + 1) * rows) <= budget:
        k += 1
    return k


def size_keys_per_pod(keys_per_pod, dim, hidden, layers, rows,
                      hbm_bytes=None, reserve=8 << 30, per_key=0,
                      clamp=True):
    """Validate ``KEYS_PER_POD`` against HBM.  Returns the usable value.

    ``per_key`` overrides the derived per-key footprint
    (``HBM_PER_KEY_BYTES``).  With ``clamp`` the result is
    ``min(keys_per_pod, max_kpp)``, else it is returned unchanged and only a
    warning is logged."""
    hbm = hbm_bytes or device_hbm_bytes()
    limit = _fit(hbm - reserve, dim, hidden, layers, rows, per_key)
    if keys_per_pod > limit:
        logger.warning('KEYS_PER_POD=%d does not fit in %.1f GB HBM '
                       '(weights %.2f GB, %.2f GB per key, max %d)%s',
                       keys_per_pod, hbm / 1e9,
                       model_bytes(dim, hidden, layers) / 1e9,
                       (per_key or per_key_bytes(rows, dim, hidden)) / 1e9,
                       limit, '; clamping' if clamp else '')
        if clamp:
            return int(max(1, limit))
    return int(keys_per_pod)


def size_from_free(keys_per_pod, free_bytes, dim, hidden, layers, rows,
                   reserve=1 << 30, per_key=0):
    """``KEYS_PER_POD`` against the HBM a standby *measured* free
    (``hipMemGetInfo`` after its HIP context, code objects and communicator
    exist, so their overhead is already excluded): the most keys whose
    engine -- weights, activations, split-K workspace -- fits in
    ``free - reserve``.  ``reserve`` covers what is allocated beyond the
    engine (graph execs, allocator slack).  Returns ``(usable kpp,
    max_kpp)``; usable is at least 1 (a worker always takes one key)."""
    limit = int(_fit(int(free_bytes) - reserve, dim, hidden, layers, rows,
                     per_key))
    return int(max(1, min(int(keys_per_pod), limit))), limit


def report(dim, hidden, layers, rows, hbm_bytes=None, reserve=8 << 30):
    hbm = hbm_bytes or device_hbm_bytes()
    return {'hbm_bytes': hbm, 'reserve_bytes': reserve,
            'weights_bytes': model_bytes(dim, hidden, layers),
            'per_key_bytes': per_key_bytes(rows, dim, hidden),
            'engine_bytes_one_key': engine_bytes(dim, hidden, layers, rows),
            'max_keys_per_pod': int(_fit(hbm - reserve, dim, hidden, layers,
                                         rows, 0)),
            'pid': os.getpid()}
