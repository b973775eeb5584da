"""GPU worker runtime: standby pool member -> pinned worker."""
from .runtime import (QueueConsumer, WorkerConfig, WorkerRuntime,
                      apply_assignment_env)

__all__ = ['QueueConsumer', 'WorkerConfig', 'WorkerRuntime',
           'apply_assignment_env']
