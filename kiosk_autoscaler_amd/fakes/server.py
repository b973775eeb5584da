"""A small threaded RESP server in front of :class:`RedisEngine`.

Used where a *socket* is required but the native ``kredis-server``
(``csrc/kredis``) is not built (pure-CPU test runs): worker processes and the
autoscaler live in different processes and need a real endpoint (SURVEY §2.4
N8).  One thread per client keeps blocking list moves (``BLMOVE``) simple.
"""
import socket
import socketserver
import threading

from ..redisq.resp import NOT_READY, RespParser, encode_reply
from .engine import DropConnection, RedisEngine, Session


class _Handler(socketserver.BaseRequestHandler):

    def handle(self):
        engine = self.server.engine
        sock = self.request
        sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        parser = RespParser(decode=False)
        session = Session()
        while not session.closed:
            try:
                data = sock.recv(65536)
            except OSError:
                return
            if not data:
                return
            parser.feed(data)
            out = []
            while True:
                command = parser.gets()
                if command is NOT_READY:
                    break
                if not isinstance(command, list):
                    # inline command ("PING\r\n") support for humans / nc
                    command = bytes(command).split()
                try:
                    reply = engine.execute(session, command)
                except DropConnection:
                    return
                out.append(encode_reply(reply))
            if out:
                try:
                    sock.sendall(b''.join(out))
                except OSError:
                    return


class _Server(socketserver.ThreadingMixIn, socketserver.TCPServer):
    daemon_threads = True
    allow_reuse_address = True


class RespServer(object):
    """Run an engine on ``host:port`` in a background thread.

    ``port=0`` picks a free port (read it back from :attr:`port`)."""

    def __init__(self, engine=None, host='127.0.0.1', port=0):
        self.engine = engine if engine is not None else RedisEngine()
        self._server = _Server((host, port), _Handler)
        self._server.engine = self.engine
        self.host, self.port = self._server.server_address[:2]
        self._thread = None

    def start(self):
        self._thread = threading.Thread(target=self._server.serve_forever,
                                        kwargs={'poll_interval': 0.05},
                                        daemon=True)
        self._thread.start()
        return self

    def stop(self):
        self._server.shutdown()
        self._server.server_close()
        if self._thread is not None:
            self._thread.join(timeout=5)

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()


def main(argv=None):
    """``python -m kiosk_autoscaler_amd.fakes.server --port 6379``"""
    import argparse
    parser = argparse.ArgumentParser(description=__doc__)
    parser.add_argument('--host', default='127.0.0.1')
    parser.add_argument('--port', type=int, default=6379)
    parser.add_argument('--redis-version', default='7.2.0',
                        help='answer as this Redis version (5.0: no '
                             'LMOVE/BLMOVE, integer blocking timeouts)')
    args = parser.parse_args(argv)
    server = RespServer(engine=RedisEngine(version=args.redis_version),
                        host=args.host, port=args.port)
    print('listening on %s:%d' % (server.host, server.port), flush=True)
    try:
        server._server.serve_forever(poll_interval=0.1)
    except KeyboardInterrupt:
        pass


if __name__ == '__main__':
    main()
