"""Worker process entry point: ``python -m kiosk_autoscaler_amd.worker.main``.

Two start modes (both spawned by :mod:`kiosk_autoscaler_amd.gpumgr`):

* **standby** (``--pin JSON``, no ``--assign``): pinned to its GPU before
  anything loads, import the native kernel module (not PyTorch), create the
  HIP context, load every code object and size the LDS ring
  (``preinit_device``), then build the engine (weights, forward and
  warm-start graphs) before the node agent starts and pays RCCL's one-time
  load.  Such a standby **holds its GPU** (the benchmark reports that time
  as ``standby_gpu_s``); with deep idle (``POOL_IDLE_RELEASE_S``) only from
  just before the tick that assigns it until just after its scale-down.
  Report ``standby`` and block on the command pipe.
* **cold** (``--assign JSON``): start immediately.  The HIP context and
  the code objects are created on a helper thread (``preinit_device``
  releases the GIL) while the main thread imports the runtime and connects
  to Redis; the engine joins it.

With the node communicator (``node_fence`` in the pin/assignment) the
process also runs a :class:`~..parallel.nodefence.NodeFenceAgent` for its
whole life, standby and worker phases alike.

After assignment the process pins itself (``HIP_VISIBLE_DEVICES`` + CPU
affinity), builds the engine and runs :class:`WorkerRuntime`.  When the
manager drains it with ``recycle`` (or a job worker finishes), it releases
the engine and reports ``recycled`` + ``standby``: the process, with its HIP
context, becomes its GPU's standby again.
"""
import argparse
import gc
import os
import sys
import threading
import time


def _die_with_parent():
    """PR_SET_PDEATHSIG: a worker must not outlive its manager."""
    try:
        import ctypes
        import signal
        libc = ctypes.CDLL(None, use_errno=True)
        libc.prctl(1, int(signal.SIGTERM), 0, 0, 0)   # PR_SET_PDEATHSIG
    except (OSError, AttributeError):
        pass


def _stack_dump_on_sigusr1():
    """``kill -USR1 <pid>`` prints every thread's Python stack to the
    worker's stderr (the manager's log): how a worker stuck in a state is
    diagnosed without a debugger."""
    try:
        import faulthandler
        import signal
        faulthandler.register(signal.SIGUSR1, all_threads=True)
    except (ImportError, AttributeError, RuntimeError, ValueError):
        pass


def _preload(backend):
    """Import everything heavy *without* touching the GPU.  The HIP worker
    needs only the native module (engine, fence): no torch import unless
    ``WORKER_IMPORT_TORCH=1`` (then torch's bundled HIP runtime is shared)."""
    t0 = time.monotonic_ns()
    if backend == 'hip':
        from ..ops import native
        native.load(torch_first=_imports_torch())
    else:
        import numpy  # noqa: F401
    return time.monotonic_ns() - t0


def _resolve_engine(backend):
    """``WORKER_ENGINE`` may be an alias (``torch-kiosk``, ``builtin``)
    when the manager did not know the backend: resolved here, before
    anything reads it."""
    value = os.environ.get('WORKER_ENGINE')
    if value:
        from ..models import engine_spec
        os.environ['WORKER_ENGINE'] = engine_spec(value, backend)


def _engine_collectives():
    """Whether the engine runs collectives of its own.  Decided WITHOUT
    importing the engine (a plug-in imported here ran before the
    GPU pin and the comgr preference, so a module-level ``torch`` import --
    or a HIP call -- initialised the runtime on the wrong device): the
    built-in engine and the known torch engines run none
    (``NO_COLLECTIVES``); any other plug-in is assumed to."""
    spec = os.environ.get('WORKER_ENGINE')
    if not spec:
        return False
    return spec not in NO_COLLECTIVES


# engines known to run no collective of their own (the fence is then the
# process's only RCCL user: one channel suffices)
NO_COLLECTIVES = frozenset([
    'kiosk_autoscaler_amd.models.torch_kiosk:TorchKioskEngine',
    'kiosk_autoscaler_amd.models.torch_engine:TorchMlpEngine',
])


def _imports_torch():
    """Torch before the native module (one HIP runtime per process):
    ``WORKER_IMPORT_TORCH``, default on for a ``WORKER_ENGINE`` plug-in
    (which may well be a PyTorch model), off for the built-in engine."""
    default = '1' if os.environ.get('WORKER_ENGINE') else '0'
    return os.environ.get('WORKER_IMPORT_TORCH', default) not in ('0', '')


def _preimport(backend):
    """Standby: import what an assignment needs, off the critical path."""
    from . import runtime  # noqa: F401
    from ..utils import events  # noqa: F401
    if backend == 'hip':
        from ..models import mlp  # noqa: F401
    spec = os.environ.get('WORKER_ENGINE')
    if spec:
        from ..models.plugin import load_factory
        try:
            load_factory(spec)
        except Exception:  # pylint: disable=broad-except
            pass   # the assignment reports it, as a failed start


# cold spawn: the helper thread opening the device (see the module doc)
_DEVICE_OPEN = {}


def _warm_torch():
    """A PyTorch plug-in's device start-up, paid before the assignment
    needs it: torch's lazy CUDA init (its own context bookkeeping, caching
    allocator) and one small bf16 GEMM, which creates the hipBLASLt handle
    and loads a GEMM code object.  Only in a process that imported torch
    (``WORKER_ENGINE``); returns stage stamps."""
    if 'torch' not in sys.modules:
        return {}
    import torch
    if not torch.cuda.is_available():
        return {}
    _torch_device(torch)
    t0 = time.monotonic_ns()
    hook = None
    spec = os.environ.get('WORKER_ENGINE')
    if spec:
        from ..models.plugin import load_factory
        try:
            hook = getattr(load_factory(spec), 'warm_device', None)
        except Exception:  # pylint: disable=broad-except
            hook = None
    if callable(hook):
        # the engine knows what its device start-up needs (the native-kernel
        # PyTorch engine: torch's context and allocator, no BLAS handle)
        hook()
    else:
        a = torch.ones(256, 256, device='cuda', dtype=torch.bfloat16)
        float((a @ a).float().sum())
    torch.cuda.synchronize()
    return {'torch_warm_start': t0, 'torch_warm_done': time.monotonic_ns()}


def _torch_device(torch):
    """``WORKER_PIN=visible``: torch's current device is this worker's GPU
    (``KIOSK_DEVICE``) on the calling thread, not ordinal 0."""
    if os.environ.get('KIOSK_DEVICE') is not None:
        from .pinning import device_ordinal
        torch.cuda.set_device(device_ordinal())


def _bind_device(mod):
    """``WORKER_PIN=visible``: the HIP current device is per thread; the
    main thread selects the worker's GPU once the device is open (the
    helper thread that opened it selected it for itself)."""
    if os.environ.get('KIOSK_DEVICE') is not None and \
            hasattr(mod, 'set_device'):
        from .pinning import device_ordinal
        mod.set_device(device_ordinal())


def _open_device_async():
    from ..ops import native
    from .pinning import device_ordinal
    mod = native.load()

    def run():
        try:
            _DEVICE_OPEN['stages'] = dict(mod.preinit_device(
                device_ordinal()))
            _DEVICE_OPEN['stages'].update(_warm_torch())
        except Exception as err:  # pylint: disable=broad-except
            # the engine's own init reports the failure
            _DEVICE_OPEN['error'] = str(err)
    thread = threading.Thread(target=run, name='device-open', daemon=True)
    _DEVICE_OPEN['thread'] = thread
    thread.start()


def _join_device_open(stage=None):
    thread = _DEVICE_OPEN.pop('thread', None)
    if thread is None:
        return
    thread.join()
    if 'error' not in _DEVICE_OPEN:
        from ..ops import native
        _bind_device(native.load())
    if stage:
        for name, t in sorted(_DEVICE_OPEN.get('stages', {}).items(),
                              key=lambda kv: kv[1]):
            stage(name, t)
        stage('device_open_joined')


_CLIENTS = {}
# the manager pipe (set in main): the engine path reports the device's PCI
# address on it once a HIP context exists
_CHANNEL = []


def _device_pci(backend, preinit=None):
    """PCI address of the device this process drives (HIP ordinal 0 under
    its HIP_VISIBLE_DEVICES pin, ``KIOSK_DEVICE`` with every managed GPU
    visible), or None before it opened a context."""
    if backend != 'hip' or not (preinit or _ENGINES):
        return None
    try:
        from ..ops import native
        from .pinning import device_ordinal
        return native.load().device_pci_bus_id(device_ordinal())
    except Exception:  # pylint: disable=broad-except
        return None


def _report_device(backend):
    """Once per process: a standby reports its device with ``standby``, a
    cold spawn with its first engine."""
    if not _CHANNEL or backend != 'hip' or \
            getattr(_CHANNEL[0], 'device_reported', False):
        return
    pci = _device_pci(backend, True)
    if pci:
        _CHANNEL[0].device_reported = True
        _CHANNEL[0].emit('device', pci=pci)
# engines kept across recycles: the recycled
# standby's next assignment with the same model finds its weights, graph
# and pass time resident and only re-runs the warm-start kernel
_ENGINES = {}


def _engine_key(backend, cfg):
    spec = os.environ.get('WORKER_ENGINE', '')
    if spec:
        return ('plugin', spec, backend, cfg.dim, cfg.hidden, cfg.layers,
                max(cfg.rows * cfg.batch, 256), cfg.seed)
    # (the CPU mock engine is cached like the HIP one: the CPU tests of the
    # recycle / HBM-tier paths exercise the same code)
    return (backend, cfg.dim, cfg.hidden, cfg.layers,
            max(cfg.rows * cfg.batch, 256), cfg.seed)


def _cached_engine(backend, cfg, stage):
    """An engine for this assignment: the cached one when the model and its
    capacity match (anything else cached is freed first), else a new one."""
    from ..models.mlp import create_engine
    key = _engine_key(backend, cfg)
    keep = True
    if key is not None and keep and key in _ENGINES and \
            getattr(_ENGINES[key], 'engine', None) is not None:
        engine = _ENGINES[key]
        engine.reused = True
        engine.cfg = cfg
        return engine
    _join_device_open(stage)
    for old in list(_ENGINES.values()):
        old.close()
    _ENGINES.clear()
    spec = os.environ.get('WORKER_ENGINE', '')
    if spec:
        from ..models.plugin import PluginEngine
        engine = PluginEngine(spec, cfg, stage)
    else:
        engine = create_engine(backend, cfg, stage)
    if key is not None and keep:
        _ENGINES[key] = engine
    _report_device(backend)
    return engine


def _prebuild_engine(backend, pin, channel):
    """A standby the manager woke for a key's arrival builds its engine
    (weights, arena, forward graph, pass time) before the assignment: the
    scale-up then finds it cached, as a recycled standby's, and READY is the
    warm-start kernel alone.  Best effort: a failure leaves the build to
    the assignment."""
    from .runtime import WorkerConfig
    spec = pin.get('prebuild') or {}
    t0 = time.monotonic_ns()
    stages = {}

    def stage(name, t=None):
        stages[name] = round(((t or time.monotonic_ns()) - t0) / 1e6, 3)
    try:
        template = {}
        if spec.get('keys_per_pod'):
            template['keys_per_pod'] = spec['keys_per_pod']
        cfg = WorkerConfig(os.environ, {
            'worker_id': 'standby', 'kind': spec.get('kind', 'deployment'),
            'slot': pin.get('slot', 0), 'gpu': pin.get('gpu', ''),
            'template': template})
        engine = _cached_engine(backend, cfg, stage)
        stage('engine_built')
        if os.environ.get('WARM_START', '1').lower() not in (
                '0', 'false', 'no', 'off'):
            engine.warmstart()
        channel.emit('prebuilt', ms=(time.monotonic_ns() - t0) / 1e6,
                     hbm_bytes=_cached_engine_bytes(), stages=stages)
    except Exception as err:  # pylint: disable=broad-except
        _drop_cached_engines()
        channel.emit('prebuilt', ms=(time.monotonic_ns() - t0) / 1e6,
                     error='%s: %s' % (type(err).__name__, err))


def _release_engine(engine):
    """End of an assignment: a cached engine stays resident (freed when the
    process exits, a different model needs the HBM, or the standby has
    been idle ``ENGINE_IDLE_RELEASE_S``)."""
    if engine is not None and engine not in _ENGINES.values():
        engine.close()


def _cached_engine_bytes():
    total = 0
    for engine in _ENGINES.values():
        size = getattr(engine, 'hbm_bytes', None)
        if callable(size):
            try:
                total += int(size())
            except Exception:  # pylint: disable=broad-except
                pass
    return total


def _drop_cached_engines():
    """Tier 1 of the standby's HBM (ENGINE_IDLE_RELEASE_S): free the kept
    engine -- weights, arena, graphs -- and keep the HIP context, code
    objects, queue and node communicator.  Returns the bytes released."""
    released = _cached_engine_bytes()
    for engine in list(_ENGINES.values()):
        engine.close()
    _ENGINES.clear()
    gc.collect()
    return released


def _process_redis(role, host=None, port=None):
    """One sentinel-aware, retrying client per role (``work``: the serving
    loop; ``events``: the event log, which other threads also write) for the
    whole process life.  A standby serves many assignments; building fresh
    clients per assignment re-probed ``SENTINEL MASTERS`` twice on every
    assign -> READY."""
    host = host or os.environ.get('REDIS_HOST', '127.0.0.1')
    port = int(port or os.environ.get('REDIS_PORT', 6379))
    key = (role, host, port)
    client = _CLIENTS.get(key)
    if client is None:
        from ..redisq import RedisClient
        client = RedisClient(host=host, port=port,
                             backoff=float(os.environ.get('REDIS_INTERVAL',
                                                          1)))
        _CLIENTS[key] = client
    return client


def _preconnect():
    """Standby boot: connect before the first assignment (best effort)."""
    try:
        _process_redis('work')
        if os.environ.get('EVENT_LOG'):
            _process_redis('events')
    except Exception:  # pylint: disable=broad-except
        _CLIENTS.clear()   # retried lazily by the first assignment


def _build_fence_factory(config):
    if config.fence in ('none', 'off', '0'):
        return None
    from ..parallel.fence import make_agent_factory
    return make_agent_factory(config)


def main(argv=None):
    parser = argparse.ArgumentParser(description=__doc__)
    parser.add_argument('--cmd-fd', type=int, default=None)
    parser.add_argument('--ev-fd', type=int, default=None)
    parser.add_argument('--backend', default='auto')
    parser.add_argument('--assign', default=None)
    parser.add_argument('--pin', default=None,
                        help='standby: JSON {gpu, slot, cpus, preinit}')
    parser.add_argument('--standalone', action='store_true',
                        help='run as a plain pod/service (no manager): '
                             'config from the environment, drain on SIGTERM')
    args = parser.parse_args(argv)
    if args.standalone:
        return _standalone(args.backend)
    _die_with_parent()
    _stack_dump_on_sigusr1()
    # ordered for the cold spawn: pin, load the native module and start
    # opening the device first; logging, the channel and the runtime
    # modules load while the helper thread creates the HIP context
    from .pinning import apply_assignment_env, parse_assignment
    backend = args.backend
    pin = parse_assignment(args.pin) if args.pin else None
    early = parse_assignment(args.assign) if args.assign else pin
    if backend == 'auto':
        backend = 'hip' if early and early.get('gpu') not in (None, '') \
            else 'cpu'
    _resolve_engine(backend)
    if backend == 'hip' and not _engine_collectives():
        # the fence is this process's only RCCL user and moves 72 bytes: one
        # channel instead of RCCL's gfx950 default of 128 holds 166 MB of
        # HBM per communicator instead of 670 MB (profiles/r2_rccl_init);
        # an engine that runs collectives of its own (``collectives = True``
        # on its factory, the default for a user plug-in) is left alone
        os.environ.setdefault('NCCL_MIN_NCHANNELS', '1')
        os.environ.setdefault('NCCL_MAX_NCHANNELS', '1')
    if early is not None:
        # pin before anything can initialise HIP (HIP_VISIBLE_DEVICES is
        # read once, at runtime init) and before the heavy imports
        apply_assignment_env({'gpu': early.get('gpu'),
                              'cpus': early.get('cpus'),
                              'visible': early.get('visible')})
    preload_ns = _preload(backend)
    if args.assign and backend == 'hip':
        _open_device_async()
    if pin and not args.assign and backend == 'hip' and \
            pin.get('preinit') == 'device' and pin.get('node_fence') and \
            os.environ.get('FENCE', 'auto') in ('auto', 'rccl'):
        # RCCL's process init in parallel with the boot below; the node
        # agent, started after the engine build, joins it
        from ..parallel.nodefence import start_early_preload
        start_early_preload()

    import logging
    logging.basicConfig(
        level=logging.INFO, stream=sys.stderr,
        format='[%(asctime)s]:[%(levelname)s]:[%(name)s]: %(message)s')
    from .channel import Channel
    channel = Channel(args.cmd_fd, args.ev_fd)
    _CHANNEL[:] = [channel]
    preinit = {}
    node = bool((early or {}).get('node_fence')) and os.environ.get(
        'FENCE', 'auto') not in ('none', 'off', '0')
    if pin and pin.get('preinit') == 'device' and backend == 'hip':
        from ..ops import native
        try:
            mod = native.load()
            from .pinning import device_ordinal
            preinit = dict(mod.preinit_device(device_ordinal()))
            if os.environ.get('KIOSK_EMBRYO_HSA_NS'):
                # ROCr was initialised while this process waited as an
                # embryo (worker/zygote.py _HsaPreinit)
                preinit['embryo_hsa_ns'] = int(
                    os.environ.pop('KIOSK_EMBRYO_HSA_NS'))
            # a PyTorch plug-in: torch's CUDA init + hipBLASLt handle too
            preinit.update(_warm_torch())
            if not node and os.environ.get('FENCE', 'auto') in ('auto',
                                                                 'rccl'):
                # RCCL's one-time init costs seconds: pay it while idle (with
                # the node communicator its first generation pays it)
                preinit['rccl_warmup_ms'] = mod.fence_warmup(60.0)
        except Exception as err:  # pylint: disable=broad-except
            channel.emit('error', message='preinit failed: %s' % err)
            return 4
    if pin is not None and not args.assign:
        _preimport(backend)
        _preconnect()
    if pin is not None and pin.get('prebuild') and not args.assign:
        # the engine (weights, graphs -- the warm-start one included) first:
        # an assignment then reaches READY with graph launches alone, which
        # an RCCL load on the node agent's thread never holds up, and the
        # agent below joins a generation only after this build
        _prebuild_engine(backend, pin, channel)
    node_agent = None
    if node:
        # a device-mode standby (HIP context open, launch handles resolved)
        # pays RCCL's one-time load on the agent thread right away
        # (the CPU stack over the fake HIP + RCCL does the same)
        fake = os.environ.get('KIOSK_NATIVE') == 'fake'
        node_agent = _start_node_agent(
            channel, backend, early.get('slot', 0),
            preload=bool(pin) and not args.assign and (
                fake or (bool(preinit) and pin.get('preinit') == 'device')))
    assignment = parse_assignment(args.assign) if args.assign else None
    recycles = 0
    # forced retirement after N recycles (test hook; 0 = never): the soak
    # shows no idle-HBM drift over 80 assignments (profiles/r3_soak), and
    # every retirement cost a shrink plus a regrow
    max_recycles = int(os.environ.get('WORKER_MAX_RECYCLES', 0)) or None
    while True:
        if assignment is None:
            assignment = _wait_for_assignment(channel, pin, preload_ns,
                                              backend, preinit)
            if assignment is None:
                code = 0
                break
            if isinstance(assignment, int):     # pinned to another GPU
                code = assignment
                break
        code, runtime = _serve(assignment, backend, channel, node_agent)
        # Recycle: a cleanly drained (or finished job) worker has released
        # its HBM, streams and communicator but keeps its HIP context and
        # loaded code objects -- it goes back to being this GPU's standby,
        # so the next scale-up on it skips the ~2 s process boot.
        if not (code == 0 and runtime.recycle and
                (max_recycles is None or recycles < max_recycles)):
            break
        recycles += 1
        # the engine's HBM is already freed: report first, collect after
        # (the collection runs while the process waits as a standby -- and
        # not at all when the manager retires it at once: ``collect``)
        channel.emit('recycled', code=code, keys_done=runtime.keys_done,
                     recycles=recycles)
        pin = {'gpu': assignment.get('gpu'), 'slot': assignment.get('slot'),
               'cpus': assignment.get('cpus'),
               'visible': assignment.get('visible')}
        assignment = _wait_for_assignment(channel, pin, preload_ns, backend,
                                          preinit, collect=True)
        if assignment is None:
            code = 0
            break
        if isinstance(assignment, int):
            code = assignment
            break
    _join_device_open()     # never exit under a running device open
    if backend == 'hip':
        try:
            from ..ops import native
            native.load().release_kept_stream()
        except Exception:  # pylint: disable=broad-except
            pass
    # The engine (HBM, streams, graphs) and the fence are released by now;
    # skip interpreter teardown (torch/HIP static destructors take ~0.5 s)
    # so the GPU slot frees promptly.
    sys.stdout.flush()
    sys.stderr.flush()
    # the manager times a retired process's exit from here to its reaping
    # (the kernel's teardown) apart from its own command to here
    channel.emit('exiting', t=time.monotonic_ns(), code=code)
    os._exit(code)


def _start_node_agent(channel, backend, slot, preload=False):
    """The process-lifetime member of the node communicator: it serves
    ``comm_*`` / ``fence`` commands from the pipe's reader thread in the
    standby and the worker phases alike."""
    from ..parallel.nodefence import (NODE_COMMANDS, NodeFenceAgent,
                                      choose_node_transport)
    transport = choose_node_transport(os.environ.get('FENCE', 'auto'),
                                      backend)
    preload = preload and transport.name == 'rccl'
    agent = NodeFenceAgent(slot, transport, channel=channel, preload=preload)
    for cmd in NODE_COMMANDS:
        channel.direct[cmd] = agent.submit
    channel.start_reader()
    # with ``preload`` the manager counts this rank in a generation once
    # it reports ``node_preloaded``
    channel.emit('node_agent', slot=slot, transport=transport.name,
                 preload=preload)
    return agent


def _standalone(backend):
    """Worker as a Kubernetes pod (``GPUMGR=k8s``) or any supervisor: the
    GPU is whatever the device plugin exposed, the worker id is the pod's
    hostname (the kiosk consumer convention for ``processing-<q>:<host>``),
    SIGTERM (a scale-down) finishes the in-flight key and exits 0, and a
    ``job`` worker exits when the queue is empty."""
    import signal
    import socket
    import logging
    logging.basicConfig(
        level=logging.INFO, stream=sys.stderr,
        format='[%(asctime)s]:[%(levelname)s]:[%(name)s]: %(message)s')
    from .channel import Channel
    if backend == 'auto':
        try:
            import torch
            backend = 'hip' if torch.cuda.device_count() > 0 else 'cpu'
        except ImportError:
            backend = 'cpu'
    os.environ.setdefault('FENCE', 'none')   # no manager to run epochs
    _preload(backend)
    channel = Channel(None, None)
    assignment = {
        'cmd': 'assign', 'gpu': '', 'slot': 0,
        'worker_id': os.environ.get('WORKER_ID') or socket.gethostname(),
        'kind': os.environ.get('RESOURCE_TYPE', 'deployment'),
        'template': {}, 'recycle': False}

    def on_sigterm(signum, frame):
        channel.commands.put({'cmd': 'drain', 'reason': 'SIGTERM'})
    signal.signal(signal.SIGTERM, on_sigterm)
    code, _ = _serve(assignment, backend, channel)
    sys.stdout.flush()
    sys.stderr.flush()
    return code


def _hbm_free(backend, preinit):
    """Free HBM bytes an assignment on this standby can use, or None (not
    measurable: no HIP context yet).  A recycled standby's cached engine
    counts as free: an assignment of the same model reuses it and any other
    one frees it first (it was subtracted twice, under-sizing
    KEYS_PER_POD exactly when HBM is tight).  ``MOCK_HBM_FREE_BYTES`` stands
    in on CPU for the device's free memory with nothing of ours in it."""
    cached = _cached_engine_bytes()
    mock = os.environ.get('MOCK_HBM_FREE_BYTES')
    if mock:
        measured = int(mock) - cached    # what hipMemGetInfo would say
        return measured + cached
    if backend != 'hip' or not (preinit or _ENGINES):
        return None
    try:
        from ..ops import native
        free, _total = native.load().mem_info()
        return int(free) + cached
    except Exception:  # pylint: disable=broad-except
        return None


# a recycled worker waits this long for the manager's verdict (``exit`` when
# the pool parks on that pass) before it runs the garbage collection
COLLECT_AFTER_S = 0.02


def _wait_for_assignment(channel, pin, preload_ns, backend, preinit,
                         collect=False):
    """Standby: report, then block until ``assign`` (or ``exit``/EOF).
    With ``ENGINE_IDLE_RELEASE_S`` a kept engine is freed after that long
    without an assignment (``engine_released``, with the new free HBM).
    ``collect`` (a recycled worker): run ``gc.collect`` once no command came
    within ``COLLECT_AFTER_S`` -- a worker retired at once exits without
    it (a full collection of a PyTorch process is standby GPU time)."""
    from .channel import TIMEOUT
    pci = _device_pci(backend, preinit)
    if pci:
        channel.device_reported = True
    channel.emit('standby', preload_ns=preload_ns, backend=backend,
                 preinit=preinit, hbm_free=_hbm_free(backend, preinit),
                 engine_cached=bool(_ENGINES), pci=pci)
    try:
        release_s = float(os.environ.get('ENGINE_IDLE_RELEASE_S', 0) or 0)
    except ValueError:
        release_s = 0.0
    while True:
        timeout = release_s if release_s > 0 and _ENGINES else None
        if collect:
            timeout = COLLECT_AFTER_S
        message = channel.read_command(timeout=timeout)
        if message is TIMEOUT and collect:
            collect = False
            gc.collect()
            continue
        if message is TIMEOUT:
            released = _drop_cached_engines()
            channel.emit('engine_released', released_bytes=released,
                         hbm_free=_hbm_free(backend, preinit))
            continue
        if message is None or message.get('cmd') in ('exit', 'eof'):
            return None
        if message.get('cmd') == 'prebuild':
            # a key arrived while this standby's engine was released
            # (ENGINE_IDLE_RELEASE_S): rebuild it before the assignment
            _prebuild_engine(backend, dict(pin or {},
                                           prebuild=message.get('spec')),
                             channel)
            continue
        if message.get('cmd') == 'assign':
            break
    if pin and str(message.get('gpu')) != str(pin.get('gpu')):
        channel.emit('error', message='assigned GPU %s but pinned to %s'
                     % (message.get('gpu'), pin.get('gpu')))
        return 5
    return message


def _serve(assignment, backend, channel, node_agent=None):
    """Run one assignment to completion: ``(exit code, runtime)``."""
    from .runtime import WorkerConfig, WorkerRuntime, apply_assignment_env
    apply_assignment_env(assignment)
    config = WorkerConfig(os.environ, assignment)

    from ..utils.events import EventLog

    def redis_factory():
        # sentinel-aware and retrying, like the autoscaler's own client;
        # created once per process (see _process_redis)
        return _process_redis('work', config.redis_host, config.redis_port)

    events = None
    if config.record_events:
        path = os.environ.get('EVENT_LOG') or None
        events = EventLog(path=None if path == 'redis' else path,
                          redis_client=_process_redis(
                              'events', config.redis_host,
                              config.redis_port),
                          source=config.worker_id)

    def engine_factory(cfg, stage):
        return _cached_engine(backend, cfg, stage)

    faults = None
    if os.environ.get('KIOSK_FAULTS'):
        from ..utils.faults import FaultPlan
        faults = FaultPlan.from_env(redis=redis_factory(),
                                    owner=config.worker_id)
    runtime = WorkerRuntime(config, engine_factory, channel, redis_factory,
                            fence_factory=(None if node_agent is not None
                                           else _build_fence_factory(config)),
                            event_log=events, faults=faults,
                            node_agent=node_agent,
                            engine_release=_release_engine)
    code = runtime.run()
    if events is not None:
        events.emit('worker_exit_self', worker=config.worker_id,
                    keys_done=runtime.keys_done)
        events.close()
    return code, runtime


if __name__ == '__main__':
    sys.exit(main())
