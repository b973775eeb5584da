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

#: MI355X-native additions (SURVEY §5.6 "New knobs").
EXTRA_DEFAULTS = (
    ('SCALE_POLICY', str, 'reference'),     # reference | strict
    ('SCALE_DOWN_DELAY', float, 0.0),       # strict: idle grace seconds
    ('TALLY_MODE', str, 'reference'),       # reference (LLEN+SCAN) | atomic (MULTI)
    ('FIXED_RATE', bool, False),            # tick every INTERVAL (not tick+INTERVAL)
    ('IDLE_INTERVAL', float, 0.0),          # opt-in faster poll while at 0 pods
    ('GPU_IDS', str, ''),                   # '' = all visible GPUs
    ('GPUMGR', str, 'embedded'),            # embedded | unix:<path> | k8s
    ('WORKER_MODULE', str, 'kiosk_autoscaler_amd.worker.main'),
    ('WORKER_BACKEND', str, 'auto'),        # auto | hip | cpu
    ('WARM_POOL', int, -1),                 # standby processes (-1 = MAX_PODS)
    # device (HIP context + code objects + queue) | context (HIP context
    # only: no HBM) | import (imports only)
    ('WARM_POOL_MODE', str, 'device'),
    # s with no demand after which the standbys exit (0 = keep them): the
    # node then holds no GPU, like the reference at zero replicas; a key's
    # arrival wakes the pool ahead of the scale-up tick (below); each wake
    # builds a new RCCL node communicator after the woken worker is READY
    ('POOL_IDLE_RELEASE_S', float, 600.0),
    # with POOL_IDLE_RELEASE_S: s between queue-length reads while no worker
    # runs; a new key refills a parked pool before the scale-up tick (the
    # decision still waits for the tick; 0 = wake at the scale-up only)
    ('POOL_WAKE_POLL_S', float, 0.05),
    # ... and wakes this long before the tick that will scale for the key
    # (embedded manager: the loop tells it when that is), so the woken
    # standbys hold the GPU for the lead, not the whole tick phase
    ('POOL_WAKE_LEAD_S', float, 0.75),
    # s a recycled standby keeps its engine (weights, arena, graphs; ~1.2
    # GiB of the idle GPU's 2.6) without an assignment; then it frees it and
    # keeps context, queue and node communicator (0 = keep forever)
    ('ENGINE_IDLE_RELEASE_S', float, 60.0),
    ('WARM_START', bool, True),             # run the N1 warm-start kernel
    # auto (rccl with device standbys, shm otherwise; store on CPU) | rccl
    # | shm | store | gloo | none
    ('FENCE', str, 'auto'),
    ('MODEL_DIM', int, 4096),
    ('MODEL_HIDDEN', int, 16384),
    ('MODEL_LAYERS', int, 4),
    ('ROWS_PER_KEY', int, 2048),
    ('HBM_PER_KEY_BYTES', int, 0),          # 0 = derive from the model
    ('HBM_RESERVE_BYTES', int, 8 << 30),    # static sizing (no measurement)
    ('HBM_FREE_RESERVE_BYTES', int, 1 << 30),  # sizing from measured free HBM
    ('EVENT_LOG', str, ''),                 # JSONL path | 'redis' | '' (off)
    ('TICK_KEY', str, ''),                  # publish tick times to this key
    ('STATE_TTL', int, 3600),
    # s without progress while busy -> kill (0 = off)
    ('WORKER_TIMEOUT', float, 0.0),
    # s from assignment to READY -> kill (0 = off)
    ('START_TIMEOUT', float, 0.0),
    ('WORKER_RECYCLE', bool, True),         # drained worker -> warm pool
    # spawn workers by fork() from a pre-imported zygote that holds no GPU
    # (worker/zygote.py): cold spawns skip interpreter start + imports
    ('WORKER_ZYGOTE', bool, True),
    ('FENCE_COMM', str, 'node'),            # node (persistent) | epoch
    # node communicator transport after FENCE_FALLBACK_AFTER consecutive
    # failed generations ('' = keep retrying RCCL): membership keeps being
    # fenced, over host shared memory, if RCCL cannot build the node
    # communicator
    ('FENCE_FALLBACK', str, 'shm'),
    ('FENCE_FALLBACK_AFTER', int, 2),
    # s a node-communicator generation (or shrink) may take to connect; a
    # hung first init falls back within FENCE_FALLBACK_AFTER x this
    ('FENCE_INIT_TIMEOUT', float, 12.0),
    ('METRICS_PORT', int, 0),               # Prometheus /metrics port (0 = off)
    ('METRICS_ADDR', str, '0.0.0.0'),
    ('DEBUG', bool, True),
    ('LOG_FILE', str, 'autoscaler.log'),
)


class Settings(object):
    """All settings resolved once (attribute access, e.g. ``s.MAX_PODS``)."""

    def __init__(self, config=None, require_resource_name=True):
        config = config if config is not None else Config()
        self.source = config.source
        for name, cast, default in REFERENCE_DEFAULTS + EXTRA_DEFAULTS:
            if default is _MISSING and not require_resource_name:
                default = ''
            setattr(self, name, config(name, default=default, cast=cast))

    @property
    def queues(self):
        return self.QUEUES.split(self.QUEUE_DELIMITER)

    def as_dict(self):
        return {name: getattr(self, name)
                for name, _, _ in REFERENCE_DEFAULTS + EXTRA_DEFAULTS}


config = Config  # decouple-style alias: ``config()('NAME', default=..)``
