"""Worker zygote: spawn workers by ``fork()`` from a process that already
imported everything a worker needs but never touched the GPU.

A worker started from scratch pays the interpreter start and its imports
before it can open the device: ~0.1 s for the torch-free HIP worker, but
~1.5-2.2 s for a PyTorch plug-in engine (``import torch``), the dominant cost
of its cold spawn (1.89 s).  The zygote pays them once, at
manager start, and holds **no GPU** (no HIP call has been made: HIP reads
``HIP_VISIBLE_DEVICES`` at its lazy init, so each forked worker still pins
its own GPU).  A spawn is then ``fork()`` + the GPU work only.

Protocol (manager <-> zygote, one ``AF_UNIX`` ``SOCK_SEQPACKET`` pair):

* manager -> zygote: ``{"argv": [...], "env": {...}}`` with the worker's two
  pipe ends (command read end, event write end) attached as ``SCM_RIGHTS``;
* the zygote forks twice: the intermediate child exits at once, so the
  worker is re-parented to the manager (``PR_SET_CHILD_SUBREAPER``) and the
  manager reaps it like any child (:class:`ForkedChild`);
* zygote -> manager: ``{"id": <request id>, "pid": <worker pid>}`` (or
  ``{"id", "error"}``).  A reply whose id is not the pending request's is a
  late answer to one the manager gave up on, and is dropped.

The worker process then runs :func:`kiosk_autoscaler_amd.worker.main.main`
with the same argv a ``subprocess`` spawn would have used.
"""
import itertools
import json
import os
import signal
import socket
import sys
import time

PR_SET_CHILD_SUBREAPER = 36
PR_SET_PDEATHSIG = 1
MAX_MSG = 1 << 20


def become_subreaper():
    """Orphaned descendants (the zygote's workers) re-parent to this
    process, so it can ``waitpid`` them.  False if the kernel refuses."""
    try:
        import ctypes
        libc = ctypes.CDLL(None, use_errno=True)
        return libc.prctl(PR_SET_CHILD_SUBREAPER, 1, 0, 0, 0) == 0
    except (OSError, AttributeError):
        return False


class ForkedChild(object):
    """``subprocess.Popen``-shaped handle of a worker the zygote forked and
    this (subreaper) process adopted."""

    def __init__(self, pid):
        self.pid = pid
        self.returncode = None

    def poll(self):
        if self.returncode is not None:
            return self.returncode
        try:
            pid, status = os.waitpid(self.pid, os.WNOHANG)
        except ChildProcessError:
            # not (or no longer) our child: alive means still running
            try:
                os.kill(self.pid, 0)
                return None
            except ProcessLookupError:
                self.returncode = 255
                return self.returncode
        if pid == 0:
            return None
        self.returncode = os.waitstatus_to_exitcode(status)
        return self.returncode

    def wait(self, timeout=None):
        deadline = None if timeout is None else time.monotonic() + timeout
        while self.poll() is None:
            if deadline is not None and time.monotonic() > deadline:
                import subprocess
                raise subprocess.TimeoutExpired(['worker', str(self.pid)],
                                                timeout)
            time.sleep(0.005)
        return self.returncode

    def send_signal(self, sig):
        if self.returncode is None:
            try:
                os.kill(self.pid, sig)
            except ProcessLookupError:
                pass

    def kill(self):
        self.send_signal(signal.SIGKILL)

    def terminate(self):
        self.send_signal(signal.SIGTERM)


class ZygoteLost(OSError):
    """A fork request was sent but not answered in time: the zygote may
    still own (and fork a worker on) the request's pipe ends, so the caller
    must retire this zygote and must not reuse those pipes."""


class ZygoteClient(object):
    """Manager side: start the zygote, fork workers from it."""

    def __init__(self, argv, env, timeout=10.0, embryos=0, rocr_embryos=0,
                 rocr_gpus=()):
        import subprocess
        self.sock, child = socket.socketpair(socket.AF_UNIX,
                                             socket.SOCK_SEQPACKET)
        env = dict(env)
        env['KIOSK_ZYGOTE_FD'] = str(child.fileno())
        self.embryos = set()        # pids of the zygote's pre-forked workers
        self.popen = subprocess.Popen(
            list(argv) + ['--zygote-fd', str(child.fileno()),
                          '--embryos', str(int(embryos)),
                          '--rocr-embryos', str(int(rocr_embryos)),
                          '--rocr-gpus', ','.join(str(g) for g in
                                                  rocr_gpus)], env=env,
            pass_fds=(child.fileno(),), close_fds=True,
            start_new_session=True)
        child.close()
        self.timeout = float(timeout)
        self.ready = False
        self.preload_s = None
        self.forks = 0
        self._ids = itertools.count(1)

    @property
    def pid(self):
        return self.popen.pid

    def alive(self):
        return self.popen.poll() is None

    def wait_ready(self, timeout=None):
        """Block until the zygote finished its imports (True) or died."""
        if self.ready:
            return True
        self.sock.settimeout(timeout if timeout is not None else self.timeout)
        try:
            data = self.sock.recv(MAX_MSG)
        except (socket.timeout, OSError):
            return False
        if not data:
            return False
        message = json.loads(data)
        self.ready = message.get('ready', False)
        self.preload_s = message.get('preload_s')
        return self.ready

    def poll_ready(self):
        """Non-blocking :meth:`wait_ready`."""
        if self.ready:
            return True
        self.sock.setblocking(False)
        try:
            data = self.sock.recv(MAX_MSG)
        except BlockingIOError:
            return False
        except OSError:
            return False
        finally:
            self.sock.setblocking(True)
        if not data:
            return False
        message = json.loads(data)
        self.ready = message.get('ready', False)
        self.preload_s = message.get('preload_s')
        return self.ready

    def fork(self, argv, env, fds):
        """A worker process running ``worker.main.main(argv)`` with
        ``env``; ``fds`` (its pipe ends) are passed, not inherited.
        Returns a :class:`ForkedChild`."""
        if not self.ready and not self.wait_ready():
            raise OSError('zygote is not ready')
        rid = next(self._ids)
        payload = json.dumps({'id': rid, 'argv': list(argv),
                              'env': dict(env)}).encode()
        self.sock.settimeout(self.timeout)
        socket.send_fds(self.sock, [payload], list(fds))
        deadline = time.monotonic() + self.timeout
        while True:
            left = deadline - time.monotonic()
            if left <= 0:
                raise ZygoteLost('zygote did not answer fork %d in %.1f s'
                                 % (rid, self.timeout))
            self.sock.settimeout(left)
            try:
                data = self.sock.recv(MAX_MSG)
            except socket.timeout:
                continue
            except OSError as err:
                raise ZygoteLost('zygote socket failed during fork %d: %s'
                                 % (rid, err))
            if not data:
                raise ZygoteLost('zygote closed its socket during fork %d'
                                 % rid)
            reply = json.loads(data)
            if 'embryos' in reply:
                self.embryos = set(int(p) for p in reply['embryos'])
            else:
                self.embryos = set(getattr(self, 'embryos', ()))
            if reply.get('id') == rid:
                break
            # a late reply to a request given up on: not ours
        if 'pid' not in reply:
            raise OSError('zygote fork failed: %s' % reply.get('error'))
        self.forks += 1
        child = ForkedChild(int(reply['pid']))
        child.embryo = reply.get('via') == 'embryo'
        self.embryos.discard(child.pid)
        return child

    def embryo_pids(self):
        """The zygote's pre-forked workers, as last reported (reading any
        report waiting on the socket; a late fork reply read here is
        dropped, as :meth:`fork` would)."""
        while True:
            try:
                self.sock.setblocking(False)
                data = self.sock.recv(MAX_MSG)
            except (BlockingIOError, OSError):
                break
            finally:
                try:
                    self.sock.setblocking(True)
                except OSError:
                    pass
            if not data:
                break
            message = json.loads(data)
            if 'embryos' in message:
                self.embryos = set(int(p) for p in message['embryos'])
        return set(self.embryos)

    def close(self):
        self.embryo_pids()
        try:
            self.sock.close()
        except OSError:
            pass
        if self.popen.poll() is None:
            self.popen.terminate()
            try:
                self.popen.wait(timeout=5)
            except Exception:  # pylint: disable=broad-except
                self.popen.kill()
        # the embryos (this process's children) end on the zygote's EOF
        deadline = time.monotonic() + 2.0
        for pid in sorted(self.embryos):
            while True:
                try:
                    done, _ = os.waitpid(pid, os.WNOHANG)
                except ChildProcessError:
                    break
                if done or time.monotonic() > deadline:
                    break
                time.sleep(0.005)
        self.embryos = set()


# ---------------------------------------------------------------------------
# zygote process
# ---------------------------------------------------------------------------
def _preload(backend):
    """Everything a worker imports, without a single HIP call -- RCCL
    included: its dlopen registers its 573 MB fat binary, which in a process
    with a HIP context holds the runtime for ~1.1 s (5 s on a cold page
    cache) and here, before any HIP call, costs ~1 ms; every forked worker
    inherits the registration (MI355X: the child's RCCL library init 5204 ->
    26 ms, its HIP init unchanged, no thread in the zygote;
    profiles/r4_defaults/zygote_probe.jsonl)."""
    from . import main as worker_main
    worker_main._preload(backend)           # native module (+ torch)
    worker_main._preimport(backend)         # runtime, events, models, plug-in
    if backend == 'hip' and os.environ.get('FENCE', 'auto') not in (
            'none', 'off', '0', 'shm', 'store', 'gloo'):
        from ..ops import native
        try:
            native.load().fence_dlopen()
        except Exception:  # pylint: disable=broad-except
            pass    # no RCCL here: each worker's agent reports it
    from ..parallel import nodefence  # noqa: F401
    from ..redisq import RedisClient  # noqa: F401
    import logging  # noqa: F401


def _child(request, fds, sock):
    """In the grandchild: become the worker described by ``request``."""
    sock.close()
    try:
        os.setsid()
    except OSError:
        pass                    # an embryo: already a session leader
    hsa_ns = _PREINIT.settle(request)
    cmd_r, ev_w = fds
    # (a kept ROCr runtime's own descriptors: KFD, render node, events)
    keep = {0, 1, 2, cmd_r, ev_w} | _PREINIT.fds
    for fd in range(3, 1024):
        if fd not in keep:
            try:
                os.close(fd)
            except OSError:
                pass
    for sig in (signal.SIGTERM, signal.SIGINT, signal.SIGCHLD):
        signal.signal(sig, signal.SIG_DFL)
    os.environ.clear()
    os.environ.update(request['env'])
    if hsa_ns is not None:
        os.environ['KIOSK_EMBRYO_HSA_NS'] = str(hsa_ns)
    argv = list(request['argv'])
    # the fds were renumbered by SCM_RIGHTS: point the worker at them
    for flag, fd in (('--cmd-fd', cmd_r), ('--ev-fd', ev_w)):
        if flag in argv:
            argv[argv.index(flag) + 1] = str(fd)
    sys.argv = ['kiosk-worker'] + argv
    from . import main as worker_main
    try:
        code = worker_main.main(argv)
    except SystemExit as stop:
        code = stop.code if isinstance(stop.code, int) else 1
    except BaseException:  # pylint: disable=broad-except
        import traceback
        traceback.print_exc()
        code = 1
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(code or 0)


def _double_fork(body):
    """Run ``body()`` in a grandchild re-parented to the manager (the
    intermediate child exits at once; the manager is the subreaper).
    Returns the grandchild's pid, or None."""
    r, w = os.pipe()
    mid = os.fork()
    if mid == 0:
        code = 0
        try:
            os.close(r)
            intermediate = os.getpid()
            pid = os.fork()
            if pid == 0:
                os.close(w)
                # wait for the intermediate to exit: the worker is then the
                # manager's (subreaper) child and its death signal binds there
                deadline = time.monotonic() + 5.0
                while os.getppid() == intermediate and \
                        time.monotonic() < deadline:
                    time.sleep(0.0002)
                body()
                os._exit(0)
            os.write(w, str(pid).encode())
        except BaseException:  # pylint: disable=broad-except
            code = 1
        os._exit(code)
    os.close(w)
    data = b''
    while True:
        chunk = os.read(r, 64)
        if not chunk:
            break
        data += chunk
    os.close(r)
    os.waitpid(mid, 0)
    return int(data) if data else None


def _embryo(esock, rocr=False, gpu=None):
    """A pre-forked worker waiting for its request (profiles/r5_boot: the
    double ``fork`` of a torch-sized zygote, ~20 ms, was on every woken
    standby's critical path).  It holds no GPU memory and no pipe of the
    manager's until the request comes; the zygote going away ends it.
    ``rocr``: it initialises ROCr while it waits (:class:`_HsaPreinit`),
    for GPU ``gpu`` alone when given."""
    try:
        os.setsid()
    except OSError:
        pass
    keep = {0, 1, 2, esock.fileno()}
    for fd in range(3, 1024):
        if fd not in keep:
            try:
                os.close(fd)
            except OSError:
                pass
    signal.signal(signal.SIGTERM, signal.SIG_DFL)
    if rocr:
        _PREINIT.start(gpu)
    try:
        payload, fds, _flags, _addr = socket.recv_fds(esock, MAX_MSG, 4)
    except OSError:
        os._exit(0)
    if not payload or len(fds) != 2:
        os._exit(0)
    _child(json.loads(payload), fds, esock)


class _HsaPreinit(object):
    """An embryo runs ROCr's ``hsa_init`` while it waits (``--rocr-embryos``
    of them).  That is the variable part of a woken standby's HIP context --
    45-60 ms, 110-300 ms in a third of fresh processes on a busy host
    (profiles/r5_boot/context_split.jsonl) -- and HIP's own set-up after it
    is 4-11 ms: a woken boot goes from ~105 ms to ~50 ms (profiles/r5_boot).
    It maps no HBM (idle-node HBM stays 1 MiB) but opens the KFD, so it is
    one more process on the device: few of them (gpumgr/pool.py
    ``zygote_rocr_embryos``).

    ROCr reads ``ROCR_VISIBLE_DEVICES`` (and its ``HSA_*`` settings) at
    ``hsa_init``, HIP applies ``HIP_VISIBLE_DEVICES`` at ``hipInit``.  An
    embryo bound to a slot's GPU (``gpu``, the zygote's ``--rocr-gpus``)
    initialises ROCr for that device alone -- ``ROCR_VISIBLE_DEVICES=<gpu>``
    -- instead of opening every device of the node; a worker for that GPU
    then pins at the ROCr level too, so the init is kept.  At the hand-off
    the runtime is kept only if the worker's environment -- the request's,
    with its assignment's template env and pin applied -- has the same
    ``ROCR_*`` / ``HSA_*`` variables the init ran under (an
    ``HSA_*`` setting of another template was silently ignored); otherwise
    ROCr is shut down again and HIP initialises it afresh (a bound embryo
    handed another GPU's request included)."""

    # seconds an embryo waits before its init: the replacement forked right
    # after a hand-off stays clear of the woken worker's own boot
    DELAY_S = 1.0

    def __init__(self):
        self.thread = None
        self.cancel = None
        self.lib = None
        self.rocr = None
        self.gpu = None             # the slot GPU it is bound to, or None
        self.snapshot = {}          # ROCR_* / HSA_* the init runs under
        self.done_ns = None
        self.status = None          # hsa_init's, once it ran
        self.fds = set()

    def start(self, gpu=None):
        import threading
        if gpu is not None:
            self.gpu = str(gpu)
            os.environ['ROCR_VISIBLE_DEVICES'] = self.gpu
        self.rocr = os.environ.get('ROCR_VISIBLE_DEVICES')
        self.snapshot = _rocr_env(os.environ)
        self.cancel = threading.Event()
        self.thread = threading.Thread(target=self._run, daemon=True)
        self.thread.start()

    def _run(self):
        if self.cancel.wait(self.DELAY_S):
            return                  # the request came first
        try:
            import ctypes
            # the runtime the process already mapped (torch's copy in a
            # torch zygote, ROCm's otherwise), matched by soname and
            # reference-counted: HIP's own hsa_init later returns at once
            lib = ctypes.CDLL('libhsa-runtime64.so.1', mode=ctypes.RTLD_GLOBAL)
            before = _open_fds()
            status = self.status = lib.hsa_init()
            # kept even after a failed init: the thunk below ROCr caches its
            # KFD descriptor, and HIP's own init would reuse it
            self.fds = _open_fds() - before
            if status == 0:
                self.lib = lib
                self.done_ns = time.monotonic_ns()
        except (OSError, AttributeError):
            pass

    def settle(self, request):
        """At the hand-off, before the worker's environment is applied:
        the ``monotonic_ns`` stamp of a kept init, or None."""
        if self.thread is None:
            return None
        self.cancel.set()
        self.thread.join()
        if self.lib is None:
            if self.status is not None:
                self._say('hsa_init failed (%d): HIP initialises ROCr'
                          % self.status)
            return None      # (or the request came before the init)
        gpu = _request_gpu(request)
        candidate = request
        if self.gpu is not None and gpu == self.gpu:
            # the worker would pin its GPU at the ROCr level, as the init did
            candidate = dict(request, env=dict(request.get('env', {}),
                                               ROCR_VISIBLE_DEVICES=self.gpu))
        worker = _rocr_env(_worker_env(candidate))
        if worker == self.snapshot and \
                (self.gpu is None or gpu == self.gpu):
            request['env'] = candidate.get('env', {})
            return self.done_ns
        self.lib.hsa_shut_down()
        self.lib = None
        # (self.fds stay open: the thunk below ROCr keeps its KFD descriptor
        # across a shut-down and reuses it at the next init)
        self._say('ROCr shut down: the worker runs with %s (GPU %s), the '
                  'init ran with %s (GPU %s)' % (worker, gpu, self.snapshot,
                                                 self.gpu))
        return None

    @staticmethod
    def _say(text):
        sys.stderr.write('embryo %d: %s\n' % (os.getpid(), text))


_PREINIT = _HsaPreinit()


def _open_fds():
    try:
        listed = [int(fd) for fd in os.listdir('/proc/self/fd')]
    except OSError:
        return set()
    found = set()
    for fd in listed:
        try:
            os.fstat(fd)    # (not the listing's own descriptor, closed now)
            found.add(fd)
        except OSError:
            pass
    return found


def _rocr_env(env):
    """The variables ROCr reads at ``hsa_init``."""
    return {k: str(v) for k, v in env.items()
            if k.startswith(('ROCR_', 'HSA_'))}


def _request_assignment(request):
    """The ``--assign`` (else ``--pin``) payload of a fork request."""
    from .pinning import parse_assignment
    argv = list(request.get('argv', ()))
    for flag in ('--assign', '--pin'):
        if flag in argv and argv.index(flag) + 1 < len(argv):
            try:
                return parse_assignment(argv[argv.index(flag) + 1])
            except ValueError:
                return None
    return None


def _request_gpu(request):
    early = _request_assignment(request) or {}
    gpu = early.get('gpu')
    return None if gpu in (None, '') else str(gpu)


def _worker_env(request):
    """The environment the worker of ``request`` will run with: the
    request's, then its assignment's template env and GPU pin
    (worker/pinning.py), as the worker applies them before HIP starts."""
    from .pinning import apply_assignment_env
    env = {k: str(v) for k, v in request.get('env', {}).items()}
    early = _request_assignment(request)
    if early:
        apply_assignment_env({'gpu': early.get('gpu'),
                              'visible': early.get('visible'),
                              'template': early.get('template') or {}}, env)
    return env


class _Embryos(object):
    """The zygote's stock of pre-forked workers (``--embryos``), of which
    up to ``rocr`` initialise ROCr while they wait.  With ``gpus`` (the
    slots' GPUs, ``--rocr-gpus``) each ROCr embryo is bound to one of them
    and initialises ROCr for that device only; a request goes to the embryo
    bound to its GPU, else to a plain one, else to any (which then shuts
    its ROCr down, :meth:`_HsaPreinit.settle`)."""

    def __init__(self, target, rocr=0, gpus=None):
        self.target = max(0, int(target))
        self.gpus = [str(g) for g in gpus or ()]
        self.rocr = max(0, int(rocr))
        if self.gpus:
            self.rocr = min(self.rocr, len(self.gpus))
        self.ready = []             # [(pid, socket, rocr)]; rocr: bool/gpu

    def pids(self):
        return [pid for pid, _, _ in self.ready]

    def _next_rocr(self):
        """What the next embryo initialises: False, True (unbound) or the
        GPU whose ROCr embryo is missing."""
        held = [r for _, _, r in self.ready if r]
        if len(held) >= self.rocr:
            return False
        if not self.gpus:
            return True
        missing = list(self.gpus[:self.rocr])
        for r in held:
            if r in missing:
                missing.remove(r)
        return missing[0] if missing else False

    def make(self):
        rocr = self._next_rocr()
        gpu = rocr if isinstance(rocr, str) else None
        ours, theirs = socket.socketpair(socket.AF_UNIX,
                                         socket.SOCK_SEQPACKET)
        try:
            pid = _double_fork(lambda: (ours.close(),
                                        _embryo(theirs, bool(rocr), gpu)))
        finally:
            theirs.close()
        if pid is None:
            ours.close()
            return False
        self.ready.append((pid, ours, rocr))
        return True

    def _pick(self, gpu):
        """Index of the embryo for a request on ``gpu``."""
        for i, (_, _, r) in enumerate(self.ready):
            if r is True or (r and r == gpu):
                return i           # unbound ROCr, or bound to this GPU
        for i, (_, _, r) in enumerate(self.ready):
            if not r:
                return i           # a plain embryo
        return 0                   # another GPU's: it shuts its ROCr down

    def top_up(self, sock):
        """Refill the stock, yielding to a waiting request."""
        import select
        while len(self.ready) < self.target:
            if select.select([sock], [], [], 0)[0]:
                return
            try:
                if not self.make():
                    return
            except OSError:
                return

    def hand(self, payload, fds):
        """Give the request to a waiting embryo: its pid, or None (none
        left, or every one died)."""
        gpu = None
        try:
            gpu = _request_gpu(json.loads(payload))
        except (ValueError, TypeError):
            pass
        while self.ready:
            pid, esock, _ = self.ready.pop(self._pick(gpu))
            try:
                socket.send_fds(esock, [payload], list(fds))
                return pid
            except OSError:
                continue
            finally:
                esock.close()
        return None


def _serve(sock, embryos=0, rocr_embryos=0, rocr_gpus=None):
    stock = _Embryos(embryos, rocr_embryos, rocr_gpus)
    reported = []
    while True:
        stock.top_up(sock)
        if stock.pids() != reported:
            # the manager reaps the embryos it knows of when the zygote goes
            reported = stock.pids()
            sock.send(json.dumps({'embryos': reported}).encode())
        try:
            payload, fds, _flags, _addr = socket.recv_fds(sock, MAX_MSG, 4)
        except OSError:
            return 0
        if not payload:
            return 0            # the manager went away
        request = {}
        try:
            request = json.loads(payload)
            if len(fds) != 2:
                raise ValueError('expected 2 fds, got %d' % len(fds))
        except ValueError as err:
            for fd in fds:
                os.close(fd)
            sock.send(json.dumps({'id': request.get('id'),
                                  'error': str(err)}).encode())
            continue
        pid = stock.hand(payload, fds)
        via = 'embryo'
        if pid is None:
            via = 'fork'
            pid = _double_fork(lambda: _child(request, fds, sock))
        for fd in fds:
            os.close(fd)
        if pid is not None:
            reply = {'id': request.get('id'), 'pid': pid, 'via': via}
        else:
            reply = {'id': request.get('id'), 'error': 'fork failed'}
        reply['embryos'] = reported = stock.pids()
        sock.send(json.dumps(reply).encode())


def main(argv=None):
    import argparse
    parser = argparse.ArgumentParser(description=__doc__)
    parser.add_argument('--zygote-fd', type=int, required=True)
    parser.add_argument('--backend', default='cpu')
    parser.add_argument('--embryos', type=int, default=0)
    parser.add_argument('--rocr-embryos', type=int, default=0)
    parser.add_argument('--rocr-gpus', default='',
                        help='comma list: the GPU each ROCr embryo binds to')
    args = parser.parse_args(argv)
    sock = socket.socket(fileno=args.zygote_fd)
    t0 = time.monotonic()
    try:
        _preload(args.backend)
    except Exception as err:  # pylint: disable=broad-except
        sock.send(json.dumps({'ready': False, 'error': str(err)}).encode())
        return 3
    # a worker must never outlive the manager, nor the zygote
    try:
        import ctypes
        ctypes.CDLL(None).prctl(PR_SET_PDEATHSIG, int(signal.SIGTERM), 0, 0, 0)
    except (OSError, AttributeError):
        pass
    signal.signal(signal.SIGCHLD, signal.SIG_DFL)
    sock.send(json.dumps({'ready': True,
                          'preload_s': time.monotonic() - t0}).encode())
    return _serve(sock, args.embryos, args.rocr_embryos,
                  [g for g in args.rocr_gpus.split(',') if g.strip()])


if __name__ == '__main__':
    sys.exit(main())
