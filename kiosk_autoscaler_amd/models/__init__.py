"""Worker model family: residual bf16 MLP blocks (random-init weights)."""
from .mlp import (CpuMlpEngine, HipMlpEngine, create_engine, gelu_tanh_np,
                  torch_reference)

__all__ = ['CpuMlpEngine', 'HipMlpEngine', 'create_engine', 'gelu_tanh_np',
           'torch_reference']
