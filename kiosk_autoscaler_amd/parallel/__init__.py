"""Cross-GPU coordination: the RCCL membership fence.

TP/PP/SP/EP/CP are deliberately absent: the workload is request-level
replica scaling (each GPU holds a full model replica and pulls keys
independently), exactly the reference's "replicas" (SURVEY §2.2).
"""
from .fence import (FenceAgent, FenceError, GlooTransport, RcclTransport,
                    StoreTransport, build_vector, choose_transport,
                    expected_vector)

__all__ = ['FenceAgent', 'FenceError', 'GlooTransport', 'RcclTransport',
           'StoreTransport', 'build_vector', 'choose_transport',
           'expected_vector']
