"""kiosk_autoscaler_amd -- an MI355X-native GPU-worker autoscaler.

Same configuration surface and Redis-queue semantics as
vanvalenlab/kiosk-autoscaler (package surface ``autoscaler.redis`` +
``autoscaler.Autoscaler``, reference ``autoscaler/__init__.py:30-32``), with
the Kubernetes actuator replaced by a node-local GPU/process manager that
launches PyTorch-ROCm workers pinned to individual MI355X GPUs, hand-written
gfx950 kernels (warm-start + fused MLP) and an RCCL membership fence.

Subpackages: ``redisq`` (RESP client, sentinel retry proxy), ``fakes``
(in-proc engine, RESP server), ``gpumgr`` (actuator), ``worker`` (worker
runtime), ``models`` (worker model), ``ops`` (native HIP kernels),
``parallel`` (membership fence), ``utils`` (events, logging, HBM sizing),
``bench`` (load generator, simulator, metrics).
"""
import importlib

__version__ = '0.1.0'

__all__ = ['redis', 'Autoscaler', '__version__']

# resolved on first use (PEP 562): a GPU worker imports this package for
# its runtime only and should not pay for the autoscaler and the manager
_LAZY = {'redis': ('.redisq.failover', None),
         'Autoscaler': ('.autoscaler', 'Autoscaler')}


def __getattr__(name):
    if name not in _LAZY:
        raise AttributeError('module %r has no attribute %r'
                             % (__name__, name))
    module, attr = _LAZY[name]
    value = importlib.import_module(module, __name__)
    if attr is not None:
        value = getattr(value, attr)
    globals()[name] = value
    return value
