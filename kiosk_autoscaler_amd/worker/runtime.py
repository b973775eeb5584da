"""Worker runtime: GPU attach -> weights -> warm-start -> READY -> consume.

Replaces the out-of-repo GPU pod of the reference.  The
queue protocol is the one the reference's tally assumes
(``autoscaler/autoscaler.py:64-73``): a consumer atomically moves an item
from ``<q>`` into its own ``processing-<q>:<worker-id>`` list (``LMOVE ...
RIGHT LEFT`` = FIFO with producers that ``LPUSH``), processes it, then
deletes the processing key.  While the key exists the tally counts it as
in-progress work.

Items are job-hash keys (the kiosk convention); the hash may carry
``rows`` / ``passes`` / ``seed`` for the inference and receives ``status``,
timings and a checksum of the output.  A plain string item is processed
with the configured defaults.
"""
import logging
import queue as queue_mod
import time

from ..redisq import exceptions as redis_errors
from .pinning import apply_assignment_env, parse_assignment  # noqa: F401
from ..utils import keys
from ..utils.trace import trace_range

logger = logging.getLogger('Worker')


def _env_int(env, name, default):
    try:
        return int(env.get(name, default))
    except (TypeError, ValueError):
        return default


def _env_float(env, name, default):
    try:
        return float(env.get(name, default))
    except (TypeError, ValueError):
        return default


# per-job bounds (a job hash is untrusted input)
MAX_PASSES = 10000
MAX_SERVICE_MS = 600000


class JobError(ValueError):
    """A job whose parameters cannot be served; it is marked failed."""


class WorkerConfig(object):
    def __init__(self, env, assignment):
        template = assignment.get('template', {})
        self.worker_id = assignment['worker_id']
        self.kind = assignment.get('kind', 'deployment')
        self.group = '%s/%s' % (assignment.get('namespace', 'default'),
                                assignment.get('resource', ''))
        self.slot = assignment.get('slot', 0)
        self.gpu = assignment.get('gpu', '')
        self.queues = template.get('queues') or env.get(
            'QUEUES', 'predict').split(env.get('QUEUE_DELIMITER', ','))
        self.redis_host = env.get('REDIS_HOST', '127.0.0.1')
        self.redis_port = _env_int(env, 'REDIS_PORT', 6379)
        self.keys_per_pod = max(1, int(template.get(
            'keys_per_pod', _env_int(env, 'KEYS_PER_POD', 1))))
        batch_default = self.keys_per_pod if self.kind == 'job' else 1
        self.batch = max(1, _env_int(env, 'WORKER_BATCH', batch_default))
        # MODEL=DIMxHIDDENxLAYERS (the autoscaler knob; a standalone worker
        # reads it too); the manager passes the parsed MODEL_DIM /
        # MODEL_HIDDEN / MODEL_LAYERS, which win
        dim, hidden, layers = 4096, 16384, 4
        if env.get('MODEL'):
            dim, hidden, layers = (int(v) for v in
                                   str(env['MODEL']).lower().split('x'))
        self.dim = _env_int(env, 'MODEL_DIM', dim)
        self.hidden = _env_int(env, 'MODEL_HIDDEN', hidden)
        self.layers = _env_int(env, 'MODEL_LAYERS', layers)
        self.rows = _env_int(env, 'ROWS_PER_KEY', 2048)
        self.passes = _env_int(env, 'PASSES_PER_KEY', 1)
        self.seed = _env_int(env, 'MODEL_SEED', 1234)
        self.warm_start = env.get('WARM_START', '1').lower() not in (
            '0', 'false', 'no', 'off')
        self.fence = env.get('FENCE', 'auto')
        # max ms a key's forward passes pause for an in-flight fence init
        self.fence_yield_ms = _env_float(env, 'FENCE_YIELD_MS', 0.0)
        # forward chunk size (ms) while a fence epoch is in flight (0 = off)
        self.fence_chunk_ms = _env_float(env, 'FENCE_YIELD_CHUNK_MS', 2.0)
        # how long an idle worker blocks in BLMOVE: bounds drain latency
        # (the drain command waits for it: it bounds scale-down latency;
        # kredis honours it to the millisecond)
        self.poll_block = _env_float(env, 'POLL_BLOCK_S', 0.005)
        self.job_idle_exit = _env_float(env, 'JOB_IDLE_EXIT_S', 1.0)
        self.mock_work_ms = _env_float(env, 'MOCK_WORK_MS', 0.0)
        self.record_events = env.get('WORKER_EVENTS', '1') not in ('0', '')
        self.recycle = bool(assignment.get('recycle', False))


def _unknown_command(err):
    return 'unknown command' in str(err).lower()


def _bad_timeout(err):
    # Redis < 6.0: "ERR timeout is not an integer or out of range"
    return 'timeout is not' in str(err).lower()


class QueueConsumer(object):
    """Moves items into per-worker processing keys and back out.

    The move is ``LMOVE q p RIGHT LEFT`` (Redis >= 6.2).  Against an older
    server -- the reference pins ``redis~=3.5.3``
    (``/root/reference/requirements.txt:3``), a client of the Redis 5/6.0
    era -- the first ``ERR unknown command`` switches this consumer, once,
    to the exactly equivalent ``RPOPLPUSH``; the blocking wait becomes
    ``BRPOPLPUSH``, and where the server also rejects a fractional timeout
    (Redis < 6.0) a non-blocking ``RPOPLPUSH`` poll every ``poll_block``
    seconds.  The processing-key convention the tally counts
    (``/root/reference/autoscaler/autoscaler.py:67-73``) is unchanged."""

    # blocking-wait modes, newest first
    BLOCK_MODES = ('blmove', 'brpoplpush', 'poll')

    def __init__(self, redis, worker_id, queues, poll_block=0.1):
        self.redis = redis
        self.worker_id = worker_id
        self.queues = list(queues)
        self.poll_block = poll_block
        self._rotate = 0
        self._sweep = 0
        # capability cache of this consumer's connection
        self.move_mode = 'lmove'
        self.block_mode = 'blmove'

    def processing_key(self, queue, slot=0):
        return keys.processing_key(queue, self.worker_id, slot)

    def _legacy(self, what, err):
        logger.warning('redis server rejected %s (%s): worker %s falls back '
                       'to RPOPLPUSH', what, err, self.worker_id)
        self.move_mode = 'rpoplpush'
        if self.block_mode == 'blmove':
            self.block_mode = 'brpoplpush'

    def _move(self, queue, pkey):
        if self.move_mode == 'lmove':
            try:
                return self.redis.lmove(queue, pkey, 'RIGHT', 'LEFT')
            except redis_errors.ResponseError as err:
                if not _unknown_command(err):
                    raise
                self._legacy('LMOVE', err)
        return self.redis.rpoplpush(queue, pkey)

    def _block_move(self, queue, pkey, timeout):
        if self.block_mode == 'blmove':
            try:
                return self.redis.blmove(queue, pkey, timeout, 'RIGHT',
                                         'LEFT')
            except redis_errors.ResponseError as err:
                if not _unknown_command(err):
                    raise
                self._legacy('BLMOVE', err)
        if self.block_mode == 'brpoplpush':
            try:
                return self.redis.brpoplpush(queue, pkey, timeout)
            except redis_errors.ResponseError as err:
                if not _bad_timeout(err):
                    raise
                # an integer timeout would hold a drain for >= 1 s
                logger.warning('redis server rejected a %.3f s blocking '
                               'timeout (%s): worker %s polls instead',
                               timeout, err, self.worker_id)
                self.block_mode = 'poll'
        time.sleep(timeout)
        return self._move(queue, pkey)

    def pull(self, limit=1, block=True):
        """Return up to ``limit`` ``(queue, item, processing_key)`` tuples.

        Sweeps every queue with non-blocking ``LMOVE`` first, starting one
        queue further on each call (round robin: a busy first queue cannot
        starve the others of a multi-queue resource); when all are empty,
        blocks on one queue (rotating) for ``poll_block`` seconds (``BLMOVE``
        wakes the instant a key lands on that queue; the bound keeps a drain
        command from waiting long)."""
        taken = []
        start = self._sweep % len(self.queues)
        self._sweep += 1
        for queue in self.queues[start:] + self.queues[:start]:
            while len(taken) < limit:
                pkey = self.processing_key(queue, len(taken))
                item = self._move(queue, pkey)
                if item is None:
                    break
                taken.append((queue, item, pkey))
        if taken or not block:
            return taken
        queue = self.queues[self._rotate % len(self.queues)]
        self._rotate += 1
        pkey = self.processing_key(queue, 0)
        item = self._block_move(queue, pkey, self.poll_block)
        if item is not None:
            taken.append((queue, item, pkey))
        return taken

    def queues_empty(self):
        return all(self.redis.llen(q) == 0 for q in self.queues)

    def complete(self, pkey, item=None, mapping=None):
        """Drop the in-flight key; with ``mapping``, write the job's result
        hash in the same MULTI/EXEC, so no observer (the tally, a test) sees
        a job ``done`` whose processing key still counts as work -- and one
        round trip instead of two.  A connection error falls back to the
        retrying single commands (both are idempotent)."""
        if mapping is None:
            self.redis.delete(pkey)
            return
        try:
            pipe = self.redis.pipeline(transaction=True)
            pipe.hset(item, mapping=mapping)
            pipe.delete(pkey)
            pipe.execute()
            return
        except (AttributeError, redis_errors.ConnectionError):
            pass
        self.redis.hset(item, mapping=mapping)
        self.redis.delete(pkey)


class WorkerRuntime(object):
    """Runs one assigned worker to completion.  Returns the exit code."""

    def __init__(self, config, engine_factory, channel, redis_factory,
                 fence_factory=None, event_log=None, faults=None,
                 node_agent=None, engine_release=None):
        self.config = config
        self.faults = faults
        self.engine_factory = engine_factory
        self.channel = channel
        self.redis_factory = redis_factory
        self.fence_factory = fence_factory
        self.events = event_log
        self.engine = None
        self.fence_agent = None
        # process-lifetime agent of the node communicator (not ours to close)
        self.node_agent = node_agent
        # how an assignment gives its engine back (default: close it; the
        # worker process may keep it resident for its next assignment)
        self.engine_release = engine_release or (lambda e: e.close())
        self.draining = False
        # back to the standby pool after a clean finish (manager's call:
        # set by the assignment, overridden by the drain command)
        self.recycle = bool(config.recycle)
        self.stages = {}
        self.keys_done = 0
        # membership gate: the agreement seq this assignment started after,
        # and whether a fence has included this worker since
        self._gate_base = None
        self._gate_included = False
        self.fenced_out = False

    def _stage(self, name, t=None):
        t = time.monotonic_ns() if t is None else int(t)
        self.stages[name] = t
        self.channel.emit('stage', stage=name, t=t)
        return t

    def _emit_event(self, kind, **fields):
        if self.events is not None:
            fields.setdefault('worker', self.config.worker_id)
            self.events.emit(kind, **fields)

    def _handle_commands(self):
        while True:
            try:
                message = self.channel.commands.get_nowait()
            except queue_mod.Empty:
                return
            cmd = message.get('cmd')
            if cmd == 'drain':
                self.draining = True
                self.recycle = bool(message.get('recycle', False))
            elif cmd == 'undrain':
                # the manager scaled back up before this loop noticed the
                # drain: keep serving (a no-op once the loop has exited)
                self.draining = False
            elif cmd in ('exit', 'eof'):
                self.draining = True
                self.recycle = False
            elif cmd in ('fence', 'fence_abort') and self.fence_agent:
                self.fence_agent.submit(message)

    def start(self):
        cfg = self.config
        self._stage('assigned_recv')
        self.redis = self.redis_factory()
        self.engine = self.engine_factory(cfg, self._stage)
        self._stage('weights_ready')
        info = None
        if cfg.warm_start:
            info = self.engine.warmstart()
            t_warm = self._stage('warmstart_done')
        if self.faults:
            self.faults.at_start()
        t_ready = self._stage('ready')
        self.channel.emit('ready', t=t_ready, stages=self.stages)
        if info is not None:
            # stamped at the warm start, sent after READY (an event sink
            # round trip READY need not wait for)
            self._emit_event('warmstart', t_ns=t_warm,
                             **{k: v for k, v in info.items()
                                if k != 'cu_mask'})
        self._emit_event('worker_ready', gpu=cfg.slot, t_ns=t_ready,
                         stages=self.stages)
        if self.node_agent is not None:
            self.fence_agent = self.node_agent
            agreed = self.node_agent.agreement(cfg.group)
            self._gate_base = agreed['seq'] if agreed else 0
        elif self.fence_factory is not None:
            self.fence_agent = self.fence_factory(self)
            direct = getattr(self.channel, 'direct', None)
            if direct is not None and self.fence_agent is not None:
                for cmd in ('fence', 'fence_abort'):
                    direct[cmd] = self.fence_agent.submit

    def excluded(self):
        """True once the node's agreed membership of this resource, read
        from this rank's own all-reduce result, has included this worker and
        a newer one no longer does: the manager's published active set is
        authoritative, so a worker fenced out stops taking keys (it drains
        or is told otherwise by the next fence).  The first keys before any
        fence are served ungated (the fence is off the
        first-inference critical path)."""
        if self._gate_base is None:
            return False
        agreed = self.node_agent.agreement(self.config.group)
        if not agreed or agreed['seq'] <= self._gate_base:
            return False
        inside = int(self.config.slot) in agreed['slots']
        if inside:
            self._gate_included = True
        out = self._gate_included and not inside
        if out != self.fenced_out:
            self.fenced_out = out
            self.channel.emit('fenced_out' if out else 'fenced_in',
                              seq=agreed['seq'])
            self._emit_event('worker_fenced_out' if out else
                             'worker_fenced_in', seq=agreed['seq'],
                             epoch=agreed['epoch'])
        return out

    def run(self):
        cfg = self.config
        self.channel.start_reader()
        try:
            self.start()
        except Exception as err:  # pylint: disable=broad-except
            logger.exception('worker %s failed to start', cfg.worker_id)
            self.channel.emit('error', message='%s: %s' % (
                type(err).__name__, err))
            if self.engine is not None:
                self.engine.close()   # never cache a failed start
            return 3
        consumer = QueueConsumer(self.redis, cfg.worker_id, cfg.queues,
                                 cfg.poll_block)
        idle_since = time.monotonic()
        busy = False
        try:
            while True:
                self._handle_commands()
                if self.draining:
                    break
                if self.excluded():
                    time.sleep(cfg.poll_block)
                    continue
                try:
                    items = consumer.pull(limit=cfg.batch)
                except redis_errors.ConnectionError as err:
                    logger.warning('redis unavailable (%s); retrying', err)
                    time.sleep(0.5)
                    continue
                except redis_errors.ResponseError as err:
                    # a protocol error the consumer cannot adapt to must not
                    # crash-loop the worker: report it and keep trying
                    logger.error('queue pull failed (%s); retrying', err)
                    self.channel.emit('pull_error', message=str(err)[:200])
                    time.sleep(0.5)
                    continue
                if not items:
                    if busy:
                        busy = False
                        self.channel.emit('idle')
                    if cfg.kind == 'job' and (
                            time.monotonic() - idle_since >= cfg.job_idle_exit
                            and consumer.queues_empty()):
                        logger.info('job worker %s: queue empty, exiting',
                                    cfg.worker_id)
                        break
                    continue
                if not busy:
                    busy = True
                    self.channel.emit('busy')
                with trace_range('kiosk.key'):
                    self._process(consumer, items)
                idle_since = time.monotonic()
        finally:
            if self.node_agent is None:
                for cmd in ('fence', 'fence_abort'):
                    getattr(self.channel, 'direct', {}).pop(cmd, None)
                if self.fence_agent is not None:
                    if not self.recycle:
                        # the process exits next and its exit frees the
                        # communicator: a graceful RCCL finalize (or waiting
                        # out an epoch init) here only kept the GPU alive,
                        # 0.2-2.2 s per drained worker on MI355X
                        self.fence_agent.abandon()
                    elif not self.fence_agent.close():
                        self.recycle = False  # a collective may still run
            if self.engine is not None:
                self.engine_release(self.engine)
        return 0

    def max_rows(self):
        """Rows one forward can take (the engine's preallocated capacity)."""
        engine = getattr(self.engine, 'engine', None)
        limit = getattr(engine, 'max_rows', None)
        if limit is None:
            limit = max(self.config.rows * self.config.batch, 256)
        return int(limit)

    def _job_params(self, item):
        """Inference parameters of one job hash.  Raises :class:`JobError`
        for values no engine call could honour (a poison job must fail on
        its own, not crash every worker that picks it up)."""
        params = {'rows': self.config.rows, 'passes': self.config.passes,
                  'seed': self.config.seed, 'service_ms': 0}
        try:
            fields = self.redis.hgetall(item)
        except redis_errors.ResponseError:
            fields = {}  # item is not a hash key
        for name in ('rows', 'passes', 'seed', 'service_ms'):
            if name in fields:
                try:
                    params[name] = int(fields[name])
                except ValueError:
                    raise JobError('%s=%r is not an integer' % (
                        name, fields[name]))
        limit = self.max_rows()
        if not 1 <= params['rows'] <= limit:
            raise JobError('rows=%d outside [1, %d]' % (params['rows'], limit))
        if not 1 <= params['passes'] <= MAX_PASSES:
            raise JobError('passes=%d outside [1, %d]' % (params['passes'],
                                                          MAX_PASSES))
        if not 0 <= params['service_ms'] <= MAX_SERVICE_MS:
            raise JobError('service_ms=%d outside [0, %d]' % (
                params['service_ms'], MAX_SERVICE_MS))
        return params, fields

    def _fail(self, consumer, queue, item, pkey, reason, fields=True):
        """Mark a job failed and release its processing key (no requeue)."""
        logger.warning('job %s failed: %s', item, reason)
        try:
            if fields:
                self.redis.hset(item, mapping={
                    'status': 'failed', 'reason': str(reason)[:500],
                    'worker': self.config.worker_id})
        except redis_errors.ResponseError:
            pass   # not a hash key: nothing to annotate
        consumer.complete(pkey)
        self._emit_event('key_failed', item=item, queue=queue,
                         reason=str(reason)[:200])

    def _process(self, consumer, items):
        cfg = self.config
        t_start = time.monotonic_ns()
        jobs = []
        for queue, item, pkey in items:
            try:
                params, fields = self._job_params(item)
            except JobError as err:
                self._fail(consumer, queue, item, pkey, err)
                continue
            jobs.append((queue, item, pkey, params, fields))
            self._emit_event('key_start', item=item, queue=queue, t_ns=t_start,
                             gpu=cfg.slot)
        # a batch whose rows exceed the engine's capacity runs in groups
        limit = self.max_rows()
        group, rows = [], 0
        for job in jobs:
            if group and rows + job[3]['rows'] > limit:
                self._run_group(consumer, group, t_start)
                group, rows, t_start = [], 0, time.monotonic_ns()
            group.append(job)
            rows += job[3]['rows']
        if group:
            self._run_group(consumer, group, t_start)

    def _run_group(self, consumer, jobs, t_start):
        cfg = self.config
        if self.faults:
            self.faults.before_key(self.keys_done + 1, self.engine,
                                   self.redis, agent=self.node_agent)
        if callable(getattr(self.engine, 'infer', None)):
            self._run_plugin(consumer, jobs, t_start)
            return
        rows = sum(p['rows'] for _, _, _, p, _ in jobs)
        passes = max(p['passes'] for _, _, _, p, _ in jobs)
        service_ms = max(p['service_ms'] for _, _, _, p, _ in jobs)
        if service_ms > 0:
            # a fixed per-key GPU service time (the benchmark's S): run real
            # forward passes until that much GPU time has been spent
            pause = None
            if self.fence_agent is not None and (cfg.fence_yield_ms > 0 or
                                                 cfg.fence_chunk_ms > 0):
                pause = (self.fence_agent.idle, cfg.fence_yield_ms,
                         cfg.fence_chunk_ms)
            call = lambda: self.engine.forward_for(  # noqa: E731
                rows, service_ms, jobs[0][3]['seed'], pause=pause)
        else:
            call = lambda: self.engine.forward(  # noqa: E731
                rows, passes, jobs[0][3]['seed'])
        try:
            result = call()
        except (ValueError, TypeError) as err:
            # the engine rejected the arguments (std::invalid_argument):
            # these jobs fail, the worker and its device are fine
            for queue, item, pkey, _, fields in jobs:
                self._fail(consumer, queue, item, pkey, err, bool(fields))
            return
        t_done = time.monotonic_ns()
        with trace_range('kiosk.complete'):
            self._complete(consumer, jobs, result, t_start, t_done)
        # liveness for the manager's watchdog (WORKER_TIMEOUT)
        self.channel.emit('beat', keys=self.keys_done)

    def _run_plugin(self, consumer, jobs, t_start):
        """A ``WORKER_ENGINE`` batch: the engine maps the job hashes to
        result fields (models/plugin.py)."""
        batch = [{'item': item, 'queue': queue, 'rows': p['rows'],
                  'seed': p['seed'], 'passes': p['passes'],
                  'service_ms': p['service_ms'], 'fields': dict(fields)}
                 for queue, item, _, p, fields in jobs]
        try:
            outputs, ms = self.engine.infer(batch)
        except (ValueError, TypeError) as err:
            for queue, item, pkey, _, fields in jobs:
                self._fail(consumer, queue, item, pkey, err, bool(fields))
            return
        t_done = time.monotonic_ns()
        with trace_range('kiosk.complete'):
            self._complete(consumer, jobs, {'ms': ms}, t_start, t_done,
                           outputs=outputs)
        self.channel.emit('beat', keys=self.keys_done)

    def _complete(self, consumer, jobs, result, t_start, t_done,
                  outputs=None):
        cfg = self.config
        for index, (queue, item, pkey, params, fields) in enumerate(jobs):
            mapping = None
            if fields:      # results go into the job hash (kiosk convention)
                mapping = {
                    'status': 'done', 'worker': cfg.worker_id,
                    'gpu': cfg.slot, 'compute_ms': '%.3f' % result['ms'],
                    'started_ns': t_start, 'finished_ns': t_done}
                if outputs is None:
                    mapping['checksum'] = '%.6e' % result.get('checksum',
                                                              0.0)
                else:
                    mapping.update({str(k): str(v) for k, v in
                                    outputs[index].items()})
            consumer.complete(pkey, item, mapping)
            self.keys_done += 1
            self._emit_event('key_done', item=item, queue=queue, t_ns=t_done,
                             gpu=cfg.slot, compute_ms=result['ms'],
                             paused_ms=result.get('paused_ms', 0.0),
                             batch=len(jobs))
