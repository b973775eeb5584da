"""Out-of-process GPU manager: JSON-lines API over a Unix socket.

``python -m kiosk_autoscaler_amd.gpumgr.daemon --socket PATH`` runs a
:class:`GpuManager` configured from the environment (same variables as the
autoscaler) so workers outlive an autoscaler crash -- the reference's
"crash-only" recovery (``scale.py:104-106``) then costs nothing: the
restarted autoscaler reconnects and keeps managing the same workers, the way
a restarted reference autoscaler finds its Deployment still running.

Requests: ``{"op": "list", "kind": ..., "namespace": ...}``,
``{"op": "patch", "kind", "name", "namespace", "body"}``,
``{"op": "register", "kind", "namespace", "name", "template"}``,
``{"op": "status"}``, ``{"op": "tick", "t": <monotonic s>}`` (the
client's next tick, for the arrival wake).  Replies: ``{"ok": true, ...}`` or
``{"ok": false, "status": int, "reason": str}``.
"""
import argparse
import json
import logging
import os
import socket
import socketserver
import threading

from .controller import WorkerTemplate
from .resources import ActuatorError, ResourceList, ResourceView

logger = logging.getLogger('GpuManagerTransport')


def handle_request(manager, request):
    op = request.get('op')
    try:
        if op == 'list':
            kind = request['kind']
            listing = (manager.list_namespaced_deployment
                       if kind == 'deployment' else
                       manager.list_namespaced_job)(request['namespace'])
            return {'ok': True, 'items': [i.to_dict() for i in listing.items]}
        if op == 'patch':
            kind = request['kind']
            patch = (manager.patch_namespaced_deployment
                     if kind == 'deployment' else
                     manager.patch_namespaced_job)
            view = patch(request['name'], request['namespace'],
                         request['body'])
            return {'ok': True, 'item': view.to_dict()}
        if op == 'register':
            # several autoscalers (one per consumer, as kiosk deploys them)
            # can share this node's GPUs: each registers its own resource
            template = WorkerTemplate(**request['template'])
            if template.backend == 'auto':
                from . import resolve_backend
                template.backend = resolve_backend('auto', manager.slots)
            if template.backend == 'hip':
                _size_for_hbm(template)
            view = manager.register(request['kind'], request['namespace'],
                                    request['name'], template)
            return {'ok': True, 'item': view.to_dict()}
        if op == 'status':
            return {'ok': True, 'status': manager.status()}
        if op == 'tick':
            manager.note_next_tick(float(request['t']))
            return {'ok': True}
        return {'ok': False, 'status': 400, 'reason': 'unknown op %r' % op}
    except ActuatorError as err:
        return {'ok': False, 'status': err.status, 'reason': err.reason}
    except (KeyError, TypeError, ValueError) as err:
        return {'ok': False, 'status': 400, 'reason': str(err)}


def _size_for_hbm(template):
    """Clamp a remotely registered template's KEYS_PER_POD to HBM, as
    ``build_manager`` does for the daemon's own resource."""
    from ..utils import hbm
    env = template.env

    def num(name, default):
        try:
            return int(env.get(name, default))
        except (TypeError, ValueError):
            return default
    kpp = hbm.size_keys_per_pod(
        template.keys_per_pod, num('MODEL_DIM', 4096),
        num('MODEL_HIDDEN', 16384), num('MODEL_LAYERS', 4),
        num('ROWS_PER_KEY', 2048),
        reserve=num('HBM_RESERVE_BYTES', 8 << 30),
        per_key=num('HBM_PER_KEY_BYTES', 0))
    template.keys_per_pod = kpp
    env['KEYS_PER_POD'] = kpp


class _Handler(socketserver.StreamRequestHandler):
    def handle(self):
        for line in self.rfile:
            if not line.strip():
                continue
            try:
                request = json.loads(line)
            except ValueError:
                reply = {'ok': False, 'status': 400, 'reason': 'bad json'}
            else:
                reply = handle_request(self.server.manager, request)
            self.wfile.write((json.dumps(reply) + '\n').encode())
            self.wfile.flush()


class _UnixServer(socketserver.ThreadingMixIn,
                  socketserver.UnixStreamServer):
    daemon_threads = True


class ManagerServer(object):
    def __init__(self, manager, path):
        if os.path.exists(path):
            os.unlink(path)
        self.path = path
        self.manager = manager
        self._server = _UnixServer(path, _Handler)
        self._server.manager = manager
        self._thread = None

    def start(self):
        self._thread = threading.Thread(target=self._server.serve_forever,
                                        kwargs={'poll_interval': 0.1},
                                        daemon=True)
        self._thread.start()
        return self

    def stop(self):
        self._server.shutdown()
        self._server.server_close()
        try:
            os.unlink(self.path)
        except OSError:
            pass


class GpuManagerClient(object):
    """Client with the same four calls as the in-process manager."""

    def __init__(self, path, timeout=30.0):
        self.path = path
        self.timeout = timeout
        self._sock = None
        self._file = None
        self._lock = threading.Lock()

    def _call(self, request):
        with self._lock:
            for attempt in (0, 1):
                try:
                    if self._sock is None:
                        sock = socket.socket(socket.AF_UNIX,
                                             socket.SOCK_STREAM)
                        sock.settimeout(self.timeout)
                        sock.connect(self.path)
                        self._sock, self._file = sock, sock.makefile('rb')
                    self._sock.sendall((json.dumps(request) + '\n').encode())
                    line = self._file.readline()
                    if not line:
                        raise OSError('manager closed the connection')
                    break
                except OSError as err:
                    self.close()
                    if attempt:
                        raise ActuatorError(503, 'GPU manager unavailable: %s'
                                            % err)
        reply = json.loads(line)
        if not reply.get('ok'):
            raise ActuatorError(reply.get('status', 500),
                                reply.get('reason', ''))
        return reply

    def close(self):
        if self._sock is not None:
            try:
                self._sock.close()
            except OSError:
                pass
        self._sock = self._file = None

    def _list(self, kind, namespace):
        reply = self._call({'op': 'list', 'kind': kind,
                            'namespace': namespace})
        return ResourceList(items=[ResourceView.from_dict(i)
                                   for i in reply['items']])

    def list_namespaced_deployment(self, namespace):
        return self._list('deployment', namespace)

    def list_namespaced_job(self, namespace):
        return self._list('job', namespace)

    def _patch(self, kind, name, namespace, body):
        reply = self._call({'op': 'patch', 'kind': kind, 'name': name,
                            'namespace': namespace, 'body': body})
        return ResourceView.from_dict(reply['item'])

    def patch_namespaced_deployment(self, name, namespace, body):
        return self._patch('deployment', name, namespace, body)

    def patch_namespaced_job(self, name, namespace, body):
        return self._patch('job', name, namespace, body)

    def note_next_tick(self, t_monotonic):
        """Tell the daemon when this autoscaler ticks next (arrival wake,
        ``POOL_WAKE_LEAD_S``).  Best effort: an unreachable daemon must not
        end the reconcile loop -- the next list/patch reports that."""
        try:
            self._call({'op': 'tick', 't': float(t_monotonic)})
        except ActuatorError:
            pass

    def register(self, kind, namespace, name, template):
        reply = self._call({'op': 'register', 'kind': kind,
                            'namespace': namespace, 'name': name,
                            'template': template.to_dict()})
        return ResourceView.from_dict(reply['item'])

    def status(self):
        return self._call({'op': 'status'})['status']


def main(argv=None):
    from ..config import Settings
    from ..utils.logs import initialize_logger
    from . import build_manager
    parser = argparse.ArgumentParser(description=__doc__)
    parser.add_argument('--socket', default='/tmp/kiosk-gpumgr.sock')
    parser.add_argument('--status', action='store_true',
                        help='print the running daemon\'s status (slots, '
                             'standbys, resources, workers) as JSON and exit')
    args = parser.parse_args(argv)
    if args.status:
        print(json.dumps(GpuManagerClient(args.socket).status(), indent=1,
                         default=str))
        return 0
    settings = Settings(require_resource_name=False)
    initialize_logger(settings.DEBUG, log_file='')
    # the manager needs Redis for requeue, persisted state, orphan recovery
    # and the fence ids; unreachable Redis at start is fatal (crash-only,
    # like the autoscaler: the supervisor restarts the daemon)
    from ..redisq import RedisClient
    from ..utils.events import EventLog
    redis = RedisClient(host=settings.REDIS_HOST, port=settings.REDIS_PORT,
                        backoff=settings.REDIS_INTERVAL)
    if settings.EVENT_LOG == 'redis':
        events = EventLog(redis_client=redis, source='gpumgr')
    else:
        events = EventLog(path=settings.EVENT_LOG or None, source='gpumgr')
    # the autoscalers on this daemon may run other policies than its own
    # environment's: an arrival wake is deferred only under an explicit
    # SCALE_POLICY here
    manager = build_manager(
        settings, redis_client=redis, events=events,
        wake_policy=(settings.policy if os.environ.get('SCALE_POLICY')
                     else None)).start()
    if settings.METRICS_PORT:
        from ..utils import metrics
        metrics.attach(events, settings.METRICS_PORT, manager=manager,
                       addr=settings.METRICS_ADDR)
    server = ManagerServer(manager, args.socket).start()
    logger.info('GPU manager listening on %s', args.socket)
    try:
        threading.Event().wait()
    except KeyboardInterrupt:
        pass
    finally:
        server.stop()
        manager.stop()


if __name__ == '__main__':
    main()
