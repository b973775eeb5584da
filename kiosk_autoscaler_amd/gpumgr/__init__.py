"""Node-local GPU/process manager (replaces the reference's k8s layer).

``connect()`` is the ``kubernetes.config.load_incluster_config()`` +
``AppsV1Api()`` analog (reference ``autoscaler/autoscaler.py:79-87``): it
returns the actuator the Autoscaler talks to -- the process-wide embedded
manager, or a client for an out-of-process daemon (``GPUMGR=unix:PATH``).
"""
import os
import tempfile

from .controller import GpuManager, WorkerTemplate
from .daemon import GpuManagerClient, ManagerServer
from .gpus import GpuSlot, discover
from .resources import ActuatorError, ResourceList, ResourceView

_EMBEDDED = None


def set_embedded(manager):
    global _EMBEDDED
    _EMBEDDED = manager


def connect(address=None):
    """The actuator for ``GPUMGR``: ``embedded`` (this process's manager),
    ``unix:<path>`` (the manager daemon) or ``k8s`` / ``k8s-kubeconfig``
    (the Kubernetes API, like the reference)."""
    address = address or os.environ.get('GPUMGR', 'embedded')
    if address.startswith('unix:'):
        return GpuManagerClient(address[len('unix:'):])
    if address in ('k8s', 'k8s-kubeconfig'):
        from .k8s import KubernetesActuator
        return KubernetesActuator(in_cluster=address == 'k8s')
    if _EMBEDDED is None:
        raise ActuatorError(503, 'no embedded GPU manager is running')
    return _EMBEDDED


def resolve_backend(requested, slots):
    if requested in ('hip', 'cpu'):
        return requested
    return 'hip' if any(s.kind == 'gpu' for s in slots) else 'cpu'


def comgr_cache_env(environ=None):
    """Where a worker's HIP runtime caches its blit-kernel build.

    Every HIP process compiles the runtime's blit kernels through comgr at
    its first stream: ~150 ms cold, ~15-20 ms from comgr's on-disk cache
    (``$XDG_CACHE_HOME/comgr``, else ``~/.cache/comgr``;
    profiles/r4_comgr).  That is on every standby's boot, so when the
    default directory is not writable (a read-only home in a container)
    the workers get a private one under the temp dir.  Returns the env to
    add ({} when the default works or the operator chose)."""
    environ = os.environ if environ is None else environ
    if environ.get('AMD_COMGR_CACHE_DIR') or \
            environ.get('AMD_COMGR_CACHE') == '0':
        return {}
    base = environ.get('XDG_CACHE_HOME') or os.path.join(
        environ.get('HOME') or os.path.expanduser('~'), '.cache')
    default = os.path.join(base, 'comgr')
    try:
        os.makedirs(default, exist_ok=True)
        if os.access(default, os.W_OK | os.X_OK):
            return {}
    except OSError:
        pass
    fallback = os.path.join(tempfile.gettempdir(),
                            'kiosk-comgr-%d' % os.getuid())
    try:
        os.makedirs(fallback, mode=0o700, exist_ok=True)
    except OSError:
        return {}
    return {'AMD_COMGR_CACHE_DIR': fallback}


def worker_env(settings, keys_per_pod=None, backend='hip'):
    """Environment every worker of this autoscaler inherits."""
    from ..models import engine_spec
    env = {
        'REDIS_HOST': settings.REDIS_HOST, 'REDIS_PORT': settings.REDIS_PORT,
        'REDIS_INTERVAL': settings.REDIS_INTERVAL,
        'QUEUES': settings.QUEUES, 'QUEUE_DELIMITER': settings.QUEUE_DELIMITER,
        'KEYS_PER_POD': keys_per_pod or settings.KEYS_PER_POD,
        'MODEL_DIM': settings.MODEL_DIM, 'MODEL_HIDDEN': settings.MODEL_HIDDEN,
        'MODEL_LAYERS': settings.MODEL_LAYERS,
        'ROWS_PER_KEY': settings.ROWS_PER_KEY,
        'FENCE': settings.FENCE,
        'FENCE_INIT_TIMEOUT': settings.FENCE_INIT_TIMEOUT,
        'ENGINE_IDLE_RELEASE_S': settings.ENGINE_IDLE_RELEASE_S,
        'RESOURCE_NAMESPACE': settings.RESOURCE_NAMESPACE,
        'RESOURCE_NAME': settings.RESOURCE_NAME,
    }
    if settings.EVENT_LOG:
        env['EVENT_LOG'] = settings.EVENT_LOG
    # the manager re-sizes KEYS_PER_POD per assignment from the free HBM a
    # standby measured (utils.hbm.size_from_free)
    env['HBM_PER_KEY_BYTES'] = settings.HBM_PER_KEY_BYTES
    env['HBM_FREE_RESERVE_BYTES'] = settings.HBM_FREE_RESERVE_BYTES
    env.update(comgr_cache_env())
    # the engine (WORKER_ENGINE: torch-kiosk by default on GPU slots; ''
    # selects the built-in engine, which the worker reads as unset)
    # (the process environment wins, as for the other worker-side settings
    # passed through below)
    env['WORKER_ENGINE'] = engine_spec(
        os.environ.get('WORKER_ENGINE',
                       getattr(settings, 'WORKER_ENGINE', None)), backend)
    # worker-side settings that are not autoscaler knobs: the engine
    # plug-in, per-key work shape, and test / debugging hooks
    for passthrough in ('WORKER_IMPORT_TORCH',
                        'PASSES_PER_KEY', 'WORKER_BATCH', 'MODEL_SEED',
                        'JOB_IDLE_EXIT_S', 'POLL_BLOCK_S', 'WORKER_EVENTS',
                        'KIOSK_RCCL_LIB', 'KIOSK_FAULTS', 'KIOSK_ROCTX',
                        'KIOSK_SHM_DIR', 'KIOSK_NATIVE', 'KIOSK_TORCH_COMGR',
                        'MOCK_WORK_MS',
                        'FAKE_RCCL_DIR', 'FAKE_RCCL_MODE',
                        'FAKE_RCCL_INIT_MS', 'FAKE_RCCL_LOAD_MS',
                        'WORKER_MAX_RECYCLES',
                        'WARM_START'):
        if passthrough in os.environ:
            env[passthrough] = os.environ[passthrough]
    return env


def template_for(settings, backend=None, keys_per_pod=None):
    """The worker template (pod-template analog) of an autoscaler's
    resource, from its settings."""
    kpp = keys_per_pod or settings.KEYS_PER_POD
    backend = backend or settings.WORKER_BACKEND
    return WorkerTemplate(queues=settings.queues,
                          module=settings.WORKER_MODULE,
                          env=worker_env(settings, kpp, backend),
                          backend=backend, keys_per_pod=kpp)


def build_manager(settings, redis_client=None, events=None, slots=None,
                  extra_env=None, wake_policy='settings'):
    """Build (not start) the manager + register the configured resource.
    ``wake_policy``: the scale policy an arrival wake is checked against
    ('settings' = this process's ``SCALE_POLICY``; None = wake on any
    arrival, for a daemon whose autoscalers' policies it does not know)."""
    from ..utils import hbm
    if slots is None:
        cpu_slots = max(1, settings.MAX_PODS)
        slots = discover(settings.GPU_IDS, cpu_slots=cpu_slots)
    backend = resolve_backend(settings.WORKER_BACKEND, slots)
    if backend == 'cpu':
        slots = [s if s.kind == 'cpu' else GpuSlot(s.index, '', kind='cpu')
                 for s in slots] or [GpuSlot(i, '', kind='cpu')
                                     for i in range(max(1, settings.MAX_PODS))]
    kpp = settings.KEYS_PER_POD
    if backend == 'hip':
        kpp = hbm.size_keys_per_pod(
            kpp, settings.MODEL_DIM, settings.MODEL_HIDDEN,
            settings.MODEL_LAYERS, settings.ROWS_PER_KEY,
            reserve=settings.HBM_RESERVE_BYTES,
            per_key=settings.HBM_PER_KEY_BYTES)
    template = template_for(settings, backend, kpp)
    template.env.update(extra_env or {})
    pool = settings.WARM_POOL
    if pool < 0:
        pool = min(max(settings.MAX_PODS, 0), len(slots))
    fence = settings.FENCE not in ('none', 'off')
    manager = GpuManager(slots, redis_client=redis_client, pool_size=pool,
                         pool_template=template, events=events, fence=fence,
                         pool_mode=settings.WARM_POOL_MODE,
                         state_ttl=settings.STATE_TTL,
                         worker_timeout=settings.WORKER_TIMEOUT,
                         start_timeout=settings.START_TIMEOUT,
                         recycle=settings.WORKER_RECYCLE,
                         fence_comm=settings.FENCE_COMM,
                         pool_idle_release_s=settings.POOL_IDLE_RELEASE_S,
                         fence_fallback=settings.FENCE_FALLBACK,
                         fence_fallback_after=settings.FENCE_FALLBACK_AFTER,
                         fence_init_timeout=settings.FENCE_INIT_TIMEOUT,
                         zygote=settings.WORKER_ZYGOTE,
                         pool_wake_poll_s=settings.POOL_WAKE_POLL_S,
                         # the tick that scales for an arrival comes within
                         # INTERVAL (+ the tick itself) of it
                         pool_wake_hold_s=1.5 * float(settings.INTERVAL) + 1.0,
                         pool_wake_lead_s=settings.POOL_WAKE_LEAD_S,
                         pin_mode=settings.WORKER_PIN,
                         hw_queues=settings.WORKER_HW_QUEUES,
                         scale_policy=(getattr(settings, 'policy', None)
                                       if wake_policy == 'settings'
                                       else wake_policy))
    if settings.RESOURCE_NAME and settings.RESOURCE_TYPE in ('deployment',
                                                           'job'):
        manager.register(settings.RESOURCE_TYPE, settings.RESOURCE_NAMESPACE,
                         settings.RESOURCE_NAME, template)
    return manager


__all__ = ['GpuManager', 'WorkerTemplate', 'GpuManagerClient',
           'ManagerServer', 'GpuSlot', 'discover', 'ActuatorError',
           'ResourceList', 'ResourceView', 'connect', 'set_embedded',
           'build_manager', 'resolve_backend', 'template_for']
