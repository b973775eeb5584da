"""Managed processes of the node-local GPU manager: the worker
template (the pod-template analog), the manager <-> process pipe, a child
process (standby or worker) and a worker's bookkeeping.

Split out of ``controller.py``; the controller, the
standby pool (``pool.py``) and the fence orchestration (``fencing.py``)
share these types.
"""
import itertools
import json
import logging
import os
import sys
import time

logger = logging.getLogger('GpuManager')

STARTING, READY, DRAINING, EXITED = 'starting', 'ready', 'draining', 'exited'


class WorkerTemplate(object):
    """What to run for a resource (the pod template analog)."""

    def __init__(self, queues=('predict',), module=None, env=None,
                 python=None, backend='auto', keys_per_pod=1):
        self.queues = list(queues)
        self.module = module or 'kiosk_autoscaler_amd.worker.main'
        self.env = dict(env or {})
        self.python = python or sys.executable
        self.backend = backend
        self.keys_per_pod = int(keys_per_pod)

    def to_dict(self):
        return {'queues': self.queues, 'module': self.module,
                'env': self.env, 'backend': self.backend,
                'keys_per_pod': self.keys_per_pod}


def bare_worker(template):
    """Spawn with ``python -S``: our own HIP worker with the built-in engine,
    not importing torch (``WORKER_IMPORT_TORCH``), unless
    a plug-in engine or a torch import needs site-packages."""
    def flag(name):
        value = template.env.get(name, os.environ.get(name, '0'))
        return str(value) not in ('0', '')
    return (template.backend == 'hip' and
            template.module == 'kiosk_autoscaler_amd.worker.main' and
            not flag('WORKER_ENGINE') and    # a plug-in may need packages
            not flag('WORKER_IMPORT_TORCH'))


class Pipe(object):
    """Line-oriented JSON channel over a pair of pipe fds."""

    def __init__(self, cmd_w, ev_r):
        self.cmd_w = cmd_w
        self.ev_r = ev_r
        self._buf = b''
        os.set_blocking(ev_r, False)

    def send(self, message):
        data = (json.dumps(message) + '\n').encode()
        try:
            os.write(self.cmd_w, data)
            return True
        except OSError:
            return False

    def read_messages(self):
        out = []
        while True:
            try:
                chunk = os.read(self.ev_r, 65536)
            except BlockingIOError:
                break
            except OSError:
                chunk = b''
            if not chunk:
                out.append(None)  # EOF
                break
            self._buf += chunk
        while b'\n' in self._buf:
            line, self._buf = self._buf.split(b'\n', 1)
            if line.strip():
                try:
                    out.append(json.loads(line))
                except ValueError:
                    logger.warning('bad worker message %r', line[:200])
        return out

    def close(self):
        for fd in (self.cmd_w, self.ev_r):
            try:
                os.close(fd)
            except OSError:
                pass


class ManagedProcess(object):
    """A child process (standby or worker) and its control pipe."""

    _ids = itertools.count()

    def __init__(self, popen, pipe, role):
        self.popen = popen
        self.pipe = pipe
        self.role = role
        self.seq = next(self._ids)
        self.t_spawn = time.monotonic_ns()
        self.booted = False
        self.eof = False
        self.recycles = 0
        self.node_ok = False    # runs a node-communicator agent
        self.hbm_free = None    # free HBM bytes the standby measured
        self.woken = False      # spawned by an arrival wake (prebuilds)
        self.engine_cached = False  # standby holds a built engine
        self.standby_since = None   # monotonic s of its last 'standby'
        # readable once the process has exited: the manager's loop wakes on
        # it, so an exit is reaped (and its GPU time closed) at once rather
        # than at the next 50 ms poll
        self.pidfd = None
        pidfd_open = getattr(os, 'pidfd_open', None)
        if pidfd_open is not None and getattr(popen, 'pid', None):
            try:
                self.pidfd = pidfd_open(popen.pid)
            except OSError:
                self.pidfd = None

    @property
    def pid(self):
        return self.popen.pid

    def close(self):
        """Release the pipe and the exit fd (the process has exited)."""
        self.pipe.close()
        fd, self.pidfd = self.pidfd, None
        if fd is not None:
            try:
                os.close(fd)
            except OSError:
                pass


class Worker(object):
    __slots__ = ('id', 'resource', 'slot', 'proc', 'state', 'busy',
                 't_assigned', 't_ready', 't_exit', 'exit_code', 'from_pool',
                 'stages', 'last_beat', 'kill_reason', 'fenced_out',
                 'quarantined_at', 'pull_errors')

    def __init__(self, wid, resource, slot, proc, from_pool):
        self.id = wid
        self.resource = resource
        self.slot = slot
        self.proc = proc
        self.state = STARTING
        self.busy = False
        self.t_assigned = time.monotonic_ns()
        self.t_ready = None
        self.t_exit = None
        self.exit_code = None
        self.from_pool = from_pool
        self.stages = {}
        self.last_beat = time.monotonic()   # last sign of progress
        self.kill_reason = None
        self.fenced_out = False     # an agreed membership excluded it
        self.quarantined_at = None  # its node agent stopped answering
        self.pull_errors = 0        # queue pulls the server rejected

    def summary(self):
        return {'id': self.id, 'gpu': self.slot.index, 'pid': self.proc.pid,
                'state': self.state, 'busy': self.busy,
                'from_pool': self.from_pool, 't_assigned': self.t_assigned,
                't_ready': self.t_ready, 'stages': dict(self.stages),
                'exit_code': self.exit_code, 'killed': self.kill_reason,
                'fenced_out': self.fenced_out,
                'pull_errors': self.pull_errors}
