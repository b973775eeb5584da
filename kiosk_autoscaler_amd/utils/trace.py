"""roctx ranges from Python.

Thin front end over the native ``roctx_*`` functions of ``_kiosk_hip``
(``csrc/runtime/trace.cpp``, which dlopens the roctx library).  The worker
wraps every key it serves in a ``kiosk.key`` range; the native engine adds
``kiosk.warmstart`` / ``kiosk.graph_capture`` / ``kiosk.forward`` /
``kiosk.fence.*``.  Under ``rocprofv3 --marker-trace`` they appear next to
the kernels.  Where the extension is not loaded (CPU workers, the
autoscaler process itself, which never touches HIP) every call is a no-op;
importing this module never loads the extension.
"""
import contextlib
import sys

_MODULE = 'kiosk_autoscaler_amd.ops._kiosk_hip'


def _native():
    # only use the extension if something else already loaded it: tracing
    # must never be the reason a process initialises HIP
    mod = sys.modules.get(_MODULE)
    if mod is None or not hasattr(mod, 'roctx_push'):
        return None
    return mod


def available():
    mod = _native()
    return bool(mod is not None and mod.roctx_available())


@contextlib.contextmanager
def trace_range(name):
    mod = _native()
    if mod is None:
        yield
        return
    mod.roctx_push(name)
    try:
        yield
    finally:
        mod.roctx_pop()


def mark(name):
    mod = _native()
    if mod is not None:
        mod.roctx_mark(name)
