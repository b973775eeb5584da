"""Typed environment configuration (component C17).

The reference reads 12 variables through python-decouple
(``scale.py:74-92``).  decouple is not available, so this module provides a
small equivalent: environment first, then an optional ``.env`` /
``settings.ini`` found from the working directory upward (decouple's
``AutoConfig`` search), then the default.  A variable with no default that
is missing raises :class:`UndefinedValueError` -- ``RESOURCE_NAME`` keeps the
reference's fatal-at-startup behaviour (``scale.py:88``).

MI355X additions (all optional, with defaults) are listed in
:data:`EXTRA_DEFAULTS`.
"""
import configparser
import os

_MISSING = object()

TRUE_STRINGS = frozenset(['1', 'true', 'yes', 'y', 'on', 't'])
FALSE_STRINGS = frozenset(['0', 'false', 'no', 'n', 'off', 'f', ''])


class UndefinedValueError(Exception):
    """A required configuration value is not set anywhere."""


def cast_bool(value):
    if isinstance(value, bool):
        return value
    text = str(value).strip().lower()
    if text in TRUE_STRINGS:
        return True
    if text in FALSE_STRINGS:
        return False
    raise ValueError('Invalid truth value: %r' % value)


def number(value):
    """``int`` like the reference (``'5'`` -> 5), but accepts fractional
    values (``'0.5'``) so sub-second loops can be configured for tests."""
    try:
        return int(value)
    except ValueError:
        return float(value)


def _find_upwards(start, names):
    path = os.path.abspath(start)
    while True:
        for name in names:
            candidate = os.path.join(path, name)
            if os.path.isfile(candidate):
                return candidate
        parent = os.path.dirname(path)
        if parent == path:
            return None
        path = parent


def _read_env_file(path):
    values = {}
    with open(path) as handle:
        for line in handle:
            line = line.strip()
            if not line or line.startswith('#') or '=' not in line:
                continue
            key, value = line.split('=', 1)
            key = key.strip()
            if key.startswith('export '):
                key = key[len('export '):].strip()
            value = value.strip()
            if len(value) >= 2 and value[0] == value[-1] and value[0] in '"\'':
                value = value[1:-1]
            values[key] = value
    return values


def _read_ini_file(path):
    parser = configparser.ConfigParser()
    parser.optionxform = str
    parser.read(path)
    if parser.has_section('settings'):
        return dict(parser.items('settings'))
    return {}


class Config(object):
    """Lookup chain: ``environ`` -> repository file -> default."""

    def __init__(self, environ=None, search_path=None, use_files=True):
        self.environ = os.environ if environ is None else environ
        self.file_values = {}
        self.source = None
        if use_files:
            explicit = self.environ.get('ENV_FILE')
            path = explicit or _find_upwards(search_path or os.getcwd(),
                                             ('settings.ini', '.env'))
            if path and os.path.isfile(path):
                self.source = path
                if path.endswith('.ini'):
                    self.file_values = _read_ini_file(path)
                else:
                    self.file_values = _read_env_file(path)

    def __call__(self, option, default=_MISSING, cast=None):
        if option in self.environ:
            value = self.environ[option]
        elif option in self.file_values:
            value = self.file_values[option]
        elif default is not _MISSING:
            value = default
        else:
            raise UndefinedValueError(
                '%s not found. Declare it as envvar or define a default '
                'value.' % option)
        if cast is None or value is None:
            return value
        if cast is bool:
            return cast_bool(value)
        return cast(value)


#: The reference's configuration surface, same names/types/defaults
#: (``scale.py:74-92``, README table).  ``None`` default = required.
REFERENCE_DEFAULTS = (
    ('REDIS_HOST', str, 'redis-master'),
    ('REDIS_PORT', int, 6379),
    ('REDIS_INTERVAL', int, 1),
    ('QUEUES', str, 'predict,track'),
    ('QUEUE_DELIMITER', str, ','),
    ('INTERVAL', number, 5),
    ('RESOURCE_NAMESPACE', str, 'default'),
    ('RESOURCE_TYPE', str, 'deployment'),
    ('RESOURCE_NAME', str, _MISSING),
    ('MIN_PODS', int, 0),
    ('MAX_PODS', int, 1),
    ('KEYS_PER_POD', int, 1),
)

#: MI355X-native additions (SURVEY §5.6 "New knobs").  Round 4 pruned them
#: from 39 to 24: merged spellings (``SCALE_POLICY``
#: carries the strict policy's delay, ``MODEL`` the three model sizes,
#: ``FENCE_FALLBACK`` its threshold, ``METRICS_PORT`` its address,
#: ``WORKER_TIMEOUT`` the start bound) and former knobs that became
#: constants (:data:`CONSTANTS`).
EXTRA_DEFAULTS = (
    # reference | strict | strict:<s> (strict, a lower target applied once
    # it persisted s; plain strict: a zero target once it persisted one
    # INTERVAL, i.e. two ticks in a row, other scale-downs at once)
    ('SCALE_POLICY', str, 'reference'),
    ('TALLY_MODE', str, 'reference'),       # reference (LLEN+SCAN) | atomic (MULTI)
    ('FIXED_RATE', bool, False),            # tick every INTERVAL (not tick+INTERVAL)
    ('IDLE_INTERVAL', float, 0.0),          # opt-in faster poll while at 0 pods
    ('GPU_IDS', str, ''),                   # '' = all visible GPUs
    ('GPUMGR', str, 'embedded'),            # embedded | unix:<path> | k8s
    ('WORKER_MODULE', str, 'kiosk_autoscaler_amd.worker.main'),
    ('WORKER_BACKEND', str, 'auto'),        # auto | hip | cpu
    # the model the workers serve: torch-kiosk (PyTorch-ROCm on our gfx950
    # kernels) | builtin (torch-free) | torch-mlp | package.module:factory
    ('WORKER_ENGINE', str, 'torch-kiosk'),
    # standby processes (-1 = MAX_PODS): HIP context, code objects, queue,
    # prebuilt engine, RCCL node communicator
    ('WARM_POOL', int, -1),
    # s with no demand after which the standbys exit (0 = keep them): the
    # node then holds no GPU, like the reference at zero replicas; a key's
    # arrival wakes the pool ahead of the scale-up tick (below); each wake
    # builds a new RCCL node communicator while the woken standby waits for
    # that tick (its engine prebuilt: READY never waits on RCCL)
    ('POOL_IDLE_RELEASE_S', float, 0.01),
    # with POOL_IDLE_RELEASE_S: s between queue-length reads while no worker
    # runs; a new key refills a parked pool just before the scale-up tick
    # (the decision still waits for the tick; 0 = wake at the scale-up only)
    ('POOL_WAKE_POLL_S', float, 0.02),
    # auto (rccl with device standbys, shm otherwise; store on CPU) | rccl
    # | shm | store | gloo | none
    ('FENCE', str, 'auto'),
    ('FENCE_COMM', str, 'node'),            # node (persistent) | epoch
    # node communicator transport after N (default 2) consecutive failed
    # generations: '<transport>[:N]' ('' = keep retrying RCCL); RCCL is
    # tried again once the node is idle
    ('FENCE_FALLBACK', str, 'shm'),
    # s a warm node-communicator generation (or shrink) may take to connect;
    # a generation with a process new to RCCL gets max(60, 5 x this)
    ('FENCE_INIT_TIMEOUT', float, 12.0),
    ('MODEL', str, '4096x16384x4'),         # DIM x HIDDEN x LAYERS
    ('ROWS_PER_KEY', int, 2048),
    ('HBM_PER_KEY_BYTES', int, 0),          # 0 = derive from the model
    ('HBM_RESERVE_BYTES', int, 8 << 30),    # static sizing (no measurement)
    ('EVENT_LOG', str, ''),                 # JSONL path | 'redis' | '' (off)
    # 'busy[:start]' s: a busy worker without progress for <busy> s, or one
    # not READY <start> s after its assignment, is killed (0 / absent = off;
    # a cold PyTorch spawn can take far longer than a key: set start apart)
    ('WORKER_TIMEOUT', str, '0'),
    ('WORKER_RECYCLE', bool, True),         # drained worker -> warm pool
    # how a worker is pinned to its GPU: isolate (HIP_VISIBLE_DEVICES=<i>),
    # visible (every managed GPU visible, the device chosen in-process, so
    # RCCL sees its peers), auto (isolate; visible from the next spawns on
    # once a multi-rank generation reports a non-xGMI peer path)
    ('WORKER_PIN', str, 'auto'),
    # hardware queues per worker process (GPU_MAX_HW_QUEUES in its
    # environment; 0 = the environment's, HIP's default 4): on MI355X each
    # queue adds a fully resident 173 MB anonymous host mapping, which the
    # process's exit frees page by page; 2 exit ~11 ms faster than 4, and 1
    # would put every stream, the fence's too, in one FIFO
    # (profiles/r6_hw_queues)
    ('WORKER_HW_QUEUES', int, 2),
    ('METRICS_PORT', str, '0'),             # Prometheus [addr:]port (0 = off)
    ('LOG_FILE', str, 'autoscaler.log'),
)

#: Former knobs, now fixed (round 4).  ``Settings`` still exposes them as
#: attributes for the code that reads them.
CONSTANTS = {
    'DEBUG': True,                 # the reference always logs at DEBUG
    # standbys hold their GPU (context, queue, engine, RCCL); the context-
    # only and import-only modes were dominated by deep idle (round 4)
    'WARM_POOL_MODE': 'device',
    'STATE_TTL': 3600,             # s the persisted manager state lives
    'WARM_START': True,            # N1 always runs
    'WORKER_ZYGOTE': True,         # spawns fork from the pre-imported zygote
    'POOL_WAKE_LEAD_S': 0.75,      # cap of the adaptive wake lead
    'ENGINE_IDLE_RELEASE_S': 60.0,  # a standby frees an unused engine
    'HBM_FREE_RESERVE_BYTES': 1 << 30,  # kept free when sizing from hipMemGetInfo
}
TICK_KEY = 'kiosk:autoscaler:tick'   # published with EVENT_LOG=redis


def parse_model(spec):
    """``'4096x16384x4'`` -> ``(4096, 16384, 4)``."""
    try:
        dim, hidden, layers = (int(v) for v in str(spec).lower().split('x'))
    except ValueError:
        raise ValueError('MODEL must be DIMxHIDDENxLAYERS, got %r' % (spec,))
    if min(dim, hidden, layers) < 1:
        raise ValueError('MODEL sizes must be positive, got %r' % (spec,))
    return dim, hidden, layers


def parse_policy(spec):
    """``'strict:2.5'`` -> ``('strict', 2.5)``; ``'reference'`` ->
    ``('reference', 0.0)``."""
    name, _, delay = str(spec).partition(':')
    return name.strip() or 'reference', float(delay) if delay else 0.0


def parse_fallback(spec):
    """``'shm:3'`` -> ``('shm', 3)``; ``''`` -> ``('', 2)``."""
    name, _, after = str(spec).partition(':')
    return name.strip(), int(after) if after else 2


def parse_timeouts(spec):
    """``'30'`` -> ``(30.0, 0.0)``; ``'30:120'`` -> ``(30.0, 120.0)``: the
    busy-progress bound and the assignment -> READY bound (a
    merged bound killed slow cold starts)."""
    busy, _, start = str(spec).partition(':')
    return float(busy or 0), float(start or 0)


#: knobs of earlier rounds that no longer configure anything (merged into
#: another spelling or fixed, :data:`CONSTANTS`): set in the environment
#: they are reported at start-up instead of silently ignored
REMOVED_KNOBS = {
    'START_TIMEOUT': "WORKER_TIMEOUT='busy:start' (still honoured)",
    'SCALE_DOWN_DELAY': "SCALE_POLICY='strict:<s>'",
    'MODEL_DIM': "MODEL='DIMxHIDDENxLAYERS'",
    'MODEL_HIDDEN': "MODEL='DIMxHIDDENxLAYERS'",
    'MODEL_LAYERS': "MODEL='DIMxHIDDENxLAYERS'",
    'FENCE_FALLBACK_AFTER': "FENCE_FALLBACK='<transport>:<n>'",
    'METRICS_ADDR': "METRICS_PORT='<addr>:<port>'",
    'WARM_POOL_MODE': 'fixed: device',
    'STATE_TTL': 'fixed: 3600 s',
    'WARM_START': 'fixed: the warm-start kernel always runs',
    'WORKER_ZYGOTE': 'fixed: on',
    'POOL_WAKE_LEAD_S': 'fixed: adaptive, capped at 0.75 s',
    'ENGINE_IDLE_RELEASE_S': 'fixed: 60 s',
    'HBM_FREE_RESERVE_BYTES': 'fixed: 1 GiB',
}


def removed_knobs(environ=None):
    """``[(name, what replaced it)]`` for removed knobs set in
    ``environ``."""
    environ = os.environ if environ is None else environ
    return [(name, hint) for name, hint in sorted(REMOVED_KNOBS.items())
            if environ.get(name) not in (None, '')]


def parse_listen(spec, default_addr='0.0.0.0'):
    """``'9100'`` / ``'127.0.0.1:9100'`` -> ``(addr, port)``; port 0 = off."""
    addr, _, port = str(spec).rpartition(':')
    return addr or default_addr, int(port or 0)


class Settings(object):
    """All settings resolved once (attribute access, e.g. ``s.MAX_PODS``)."""

    def __init__(self, config=None, require_resource_name=True):
        config = config if config is not None else Config()
        self.source = config.source
        for name, cast, default in REFERENCE_DEFAULTS + EXTRA_DEFAULTS:
            if default is _MISSING and not require_resource_name:
                default = ''
            setattr(self, name, config(name, default=default, cast=cast))
        for name, value in CONSTANTS.items():
            setattr(self, name, value)
        # derived from the merged spellings
        self.MODEL_DIM, self.MODEL_HIDDEN, self.MODEL_LAYERS = \
            parse_model(self.MODEL)
        self.policy, self.SCALE_DOWN_DELAY = parse_policy(self.SCALE_POLICY)
        self.SCALE_TO_ZERO_DELAY = 0.0
        if self.policy == 'strict' and ':' not in str(self.SCALE_POLICY):
            # strict's default hysteresis, on the last workers only: a
            # target of zero must be read on two consecutive ticks before
            # they go.  Mid-burst the system empties for a tick often
            # (Poisson lam = 2/s, 1 s keys: P(no key) = e^-2 = 13.5 % per
            # tick) and a scale-down to zero there makes the next key pay a
            # cold start; two readings in a row: 1.8 %.
            # A scale-down that keeps workers applies at once (the pool
            # re-wakes standbys ahead of the tick for a new rise).
            # ``strict:<s>`` holds every scale-down <s> s; ``strict:0``
            # none.
            self.SCALE_TO_ZERO_DELAY = float(self.INTERVAL)
        self.FENCE_FALLBACK, self.FENCE_FALLBACK_AFTER = \
            parse_fallback(self.FENCE_FALLBACK)
        self.METRICS_ADDR, self.METRICS_PORT = parse_listen(self.METRICS_PORT)
        self.WORKER_TIMEOUT, self.START_TIMEOUT = parse_timeouts(
            self.WORKER_TIMEOUT)
        legacy = config('START_TIMEOUT', default='')
        if legacy not in ('', None) and ':' not in str(
                config('WORKER_TIMEOUT', default='')):
            # the round-3 knob, still honoured for its start bound
            self.START_TIMEOUT = float(legacy)
        self.TICK_KEY = TICK_KEY if self.EVENT_LOG == 'redis' else ''

    @property
    def queues(self):
        return self.QUEUES.split(self.QUEUE_DELIMITER)

    def as_dict(self):
        return {name: getattr(self, name)
                for name, _, _ in REFERENCE_DEFAULTS + EXTRA_DEFAULTS}


config = Config  # decouple-style alias: ``config()('NAME', default=..)``
