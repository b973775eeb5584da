"""GPU worker runtime: standby pool member -> pinned worker.

The names below resolve on first use (PEP 562): ``python -m
kiosk_autoscaler_amd.worker.main`` imports this package first, and a
cold-spawned worker should reach its device open before the runtime, the
Redis client and logging load (see ``main``)."""
import importlib

__all__ = ['QueueConsumer', 'WorkerConfig', 'WorkerRuntime',
           'apply_assignment_env']


def __getattr__(name):
    if name not in __all__:
        raise AttributeError('module %r has no attribute %r'
                             % (__name__, name))
    value = getattr(importlib.import_module('.runtime', __name__), name)
    globals()[name] = value
    return value
