"""Bring-your-own engine: ``WORKER_ENGINE=package.module:factory``.

The reference scales whatever consumer image its Deployment runs; here the
worker process (standby pool, GPU pinning, warm-start, queue protocol,
drain/recycle, membership fence) is the framework's, and the model is a
plug-in.  ``factory(cfg, stage)`` is called once per assignment (the result
is cached across recycles like the built-in engine) with the
:class:`~kiosk_autoscaler_amd.worker.runtime.WorkerConfig` and a
``stage(name)`` callback for start-up timestamps, and returns an object
with

* ``infer(jobs) -> list of dict`` -- one call per batch (``WORKER_BATCH``
  / ``KEYS_PER_POD`` items).  Each job is ``{'item', 'queue', 'rows',
  'seed', 'passes', 'service_ms', 'fields'}`` (``fields`` = the job hash).
  Return one dict per job: its entries are written into that job's hash
  next to ``status=done``.  Raise ``ValueError`` / ``TypeError`` for input
  the model cannot take: those jobs are marked ``failed``, the worker keeps
  serving.  Any other exception ends the worker; the manager requeues its
  in-flight items and restarts it (the built-in engine's contract).
* ``warmstart() -> dict`` (optional) -- runs before READY, e.g. one dry
  forward so the first request finds kernels loaded.
* ``close()`` (optional) -- free device memory.
* ``max_rows`` (optional attribute) -- rows one ``infer`` batch may hold.

A PyTorch engine needs torch in the worker: with ``WORKER_ENGINE`` set the
worker imports torch before the native module unless
``WORKER_IMPORT_TORCH=0`` (one HIP runtime per process), and it is spawned
with site-packages.  :mod:`.torch_engine` is a complete example on MI355X;
:class:`ReverseEngine` below is the minimal CPU one the tests use.
"""
import importlib
import time


def load_factory(spec):
    """``'package.module:callable'`` -> the callable."""
    module, sep, attr = str(spec).partition(':')
    if not sep or not module or not attr:
        raise ValueError('WORKER_ENGINE must be "package.module:callable", '
                         'got %r' % spec)
    target = importlib.import_module(module)
    for part in attr.split('.'):
        target = getattr(target, part)
    if not callable(target):
        raise TypeError('WORKER_ENGINE %r is not callable' % spec)
    return target


class PluginEngine(object):
    """Adapter between a user engine and the worker runtime."""

    name = 'plugin'

    def __init__(self, spec, cfg, stage=None):
        self.spec = spec
        self.cfg = cfg
        self.reused = False
        self.user = load_factory(spec)(cfg, stage)
        if not callable(getattr(self.user, 'infer', None)):
            raise TypeError('engine from %r has no infer(jobs)' % spec)
        self.engine = self          # the runtime reads .engine.max_rows
        limit = getattr(self.user, 'max_rows', None)
        self.max_rows = int(limit) if limit else max(cfg.rows * cfg.batch,
                                                     256)

    def warmstart(self):
        hook = getattr(self.user, 'warmstart', None)
        info = dict(hook() or {}) if callable(hook) else {}
        info.setdefault('backend', 'plugin')
        info['reused'] = self.reused
        return info

    def infer(self, jobs):
        t0 = time.perf_counter()
        outputs = self.user.infer(jobs)
        ms = (time.perf_counter() - t0) * 1e3
        outputs = list(outputs) if outputs is not None else []
        if len(outputs) != len(jobs):
            raise ValueError('engine returned %d results for %d jobs'
                             % (len(outputs), len(jobs)))
        return [dict(o or {}) for o in outputs], ms

    def hbm_bytes(self):
        """Device bytes the user engine holds (its ``hbm_bytes()``, if it
        has one): what the standby reports as released / reusable."""
        hook = getattr(self.user, 'hbm_bytes', None)
        return int(hook()) if callable(hook) else 0

    def close(self):
        user, self.user = self.user, None
        self.engine = None
        hook = getattr(user, 'close', None)
        if callable(hook):
            hook()


class ReverseEngine(object):
    """Minimal CPU example: reverses each job's ``payload`` field."""

    def __init__(self, cfg, stage=None):
        self.prefix = ''
        if stage:
            stage('device_ready')

    def warmstart(self):
        self.prefix = 'rev:'
        return {'backend': 'cpu-example'}

    def infer(self, jobs):
        out = []
        for job in jobs:
            payload = job['fields'].get('payload')
            if payload is None:
                raise ValueError('job %s has no payload' % job['item'])
            out.append({'output': self.prefix + payload[::-1]})
        return out
