"""Worker model family: residual bf16 MLP blocks (random-init weights).

Engines a worker can run (``WORKER_ENGINE``):

* ``torch-kiosk`` (default on GPU slots) -- the PyTorch-ROCm engine
  (:class:`.torch_kiosk.TorchKioskEngine`): torch tensors, torch's stream and
  native hipGraphs around the hand-written gfx950 kernels;
* ``builtin`` -- the torch-free engine of the native module
  (:class:`.mlp.HipMlpEngine`), spawned with ``python -S``;
* ``torch-mlp`` -- the plain-PyTorch example (:mod:`.torch_engine`);
* ``package.module:factory`` -- a user engine (:mod:`.plugin`).

CPU slots run the mock engine (:class:`.mlp.CpuMlpEngine`) unless a plug-in
is named explicitly.
"""
from .mlp import (CpuMlpEngine, HipMlpEngine, create_engine, gelu_tanh_np,
                  torch_reference)

#: engine aliases -> plug-in specs (``builtin``: no plug-in)
ENGINES = {
    'torch-kiosk': 'kiosk_autoscaler_amd.models.torch_kiosk:TorchKioskEngine',
    'torch-mlp': 'kiosk_autoscaler_amd.models.torch_engine:TorchMlpEngine',
    'builtin': '',
}
DEFAULT_ENGINE = 'torch-kiosk'
_BUILTIN_NAMES = ('', 'builtin', 'native', 'none')


def engine_spec(value, backend):
    """The ``WORKER_ENGINE`` a worker process gets: a plug-in spec, or ``''``
    for the built-in engine (the torch-free HIP one, or the CPU mock).
    ``value`` is the setting (an alias or ``package.module:factory``;
    ``None`` = the default)."""
    value = DEFAULT_ENGINE if value is None else str(value).strip()
    if value.lower() in _BUILTIN_NAMES:
        return ''
    if value in ENGINES:
        # the aliases are GPU engines: CPU slots keep their mock engine; an
        # undecided backend ('auto', a manager daemon's template) passes the
        # alias on and the worker resolves it once it knows its backend
        if backend == 'hip':
            return ENGINES[value]
        return value if backend == 'auto' else ''
    return value


def engine_name(spec):
    """Short name of a resolved spec (``engine_spec``) for reports."""
    for name, full in ENGINES.items():
        if spec == full:
            return name
    return spec or 'builtin'


__all__ = ['CpuMlpEngine', 'HipMlpEngine', 'create_engine', 'gelu_tanh_np',
           'torch_reference', 'ENGINES', 'DEFAULT_ENGINE', 'engine_spec',
           'engine_name']
