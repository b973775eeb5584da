"""HBM sizing for ``KEYS_PER_POD`` (BASELINE config 5).

A worker keeps its model resident in HBM and, in one-shot ``job`` mode,
batches up to ``KEYS_PER_POD`` keys into one forward pass.  This module
computes how many keys' working sets fit beside the weights on one MI355X
(288 GB HBM3E) and clamps / warns when the configured value does not fit:

    max_kpp = floor((HBM_total - reserve - weights) / per_key_bytes)

Byte counts follow the worker model (:mod:`kiosk_autoscaler_amd.models.mlp`):
bf16 weights ``L x (2*D*H + H + D)`` and, per key of ``R`` rows, the input,
the GELU hidden activation and the output (``R x (2D + H)`` bf16) plus the
fp32 row checksum.
"""
import logging
import os

MI355X_HBM_BYTES = 288 * 10 ** 9   # spec capacity (decimal GB)
BF16 = 2

logger = logging.getLogger('HbmSizing')


def model_bytes(dim, hidden, layers):
    return layers * (2 * dim * hidden + hidden + dim) * BF16


def per_key_bytes(rows, dim, hidden):
    return rows * (2 * dim + hidden) * BF16 + rows * 4


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


def size_keys_per_pod(keys_per_pod, dim, hidden, layers, rows,
                      hbm_bytes=None, reserve=8 << 30, per_key=0,
                      clamp=True):
    """Validate ``KEYS_PER_POD`` against HBM.  Returns the usable value.

    ``per_key`` overrides the derived per-key footprint
    (``HBM_PER_KEY_BYTES``).  With ``clamp`` the result is
    ``min(keys_per_pod, max_kpp)``, else it is returned unchanged and only a
    warning is logged."""
    hbm = hbm_bytes or device_hbm_bytes()
    weights = model_bytes(dim, hidden, layers)
    footprint = per_key or per_key_bytes(rows, dim, hidden)
    limit = max_keys_per_pod(hbm, weights, footprint, reserve)
    if keys_per_pod > limit:
        logger.warning('KEYS_PER_POD=%d does not fit in %.1f GB HBM '
                       '(weights %.2f GB, %.2f GB per key, max %d)%s',
                       keys_per_pod, hbm / 1e9, weights / 1e9,
                       footprint / 1e9, limit,
                       '; clamping' if clamp else '')
        if clamp:
            return int(max(1, limit))
    return int(keys_per_pod)


def size_from_free(keys_per_pod, free_bytes, dim, hidden, layers, rows,
                   reserve=1 << 30, per_key=0):
    """``KEYS_PER_POD`` against the HBM a standby *measured* free
    (``hipMemGetInfo`` after its HIP context, code objects and communicator
    exist, so their overhead is already excluded):

        max_kpp = floor((HBM_free - weights - reserve) / per_key_bytes)

    ``reserve`` covers what the engine allocates beyond weights and per-key
    activations (split-K workspace, graph exec, allocator slack).  Returns
    ``(usable kpp, max_kpp)``; usable is at least 1 (a worker always takes
    one key)."""
    weights = model_bytes(dim, hidden, layers)
    footprint = per_key or per_key_bytes(rows, dim, hidden)
    limit = int(max_keys_per_pod(int(free_bytes), weights, footprint,
                                 reserve))
    return int(max(1, min(int(keys_per_pod), limit))), limit


def report(dim, hidden, layers, rows, hbm_bytes=None, reserve=8 << 30):
    hbm = hbm_bytes or device_hbm_bytes()
    weights = model_bytes(dim, hidden, layers)
    per_key = per_key_bytes(rows, dim, hidden)
    return {'hbm_bytes': hbm, 'reserve_bytes': reserve,
            'weights_bytes': weights, 'per_key_bytes': per_key,
            'max_keys_per_pod': int(max_keys_per_pod(hbm, weights, per_key,
                                                     reserve)),
            'pid': os.getpid()}
