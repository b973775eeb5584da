"""Native MI355X ops: gfx950 HIP kernels + RCCL fence (module ``_kiosk_hip``).

Kernels (``csrc/kernels``): the N2 fused MLP GEMMs (MFMA
``v_mfma_f32_16x16x32_bf16``, LDS double-buffered via ``global_load_lds``,
fused bias/GELU/residual epilogues, XCD-aware tile order), the N1 warm-start
kernel, and on-device random weight init.  Python wrappers that take torch
tensors live in :mod:`kiosk_autoscaler_amd.ops.kernels`.
"""
from .native import NativeUnavailable, available, load

__all__ = ['NativeUnavailable', 'available', 'load']
