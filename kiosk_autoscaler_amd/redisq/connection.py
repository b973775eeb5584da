"""Blocking TCP connections and a small thread-safe pool.

Connections are lazy: nothing touches the network until the first command,
which is the behaviour the reference relies on when it constructs clients
for sentinel-discovered hosts (``autoscaler/redis.py:157-161``).
"""
import socket
import threading

from . import exceptions
from .resp import NOT_READY, RespParser, encode_command, encode_commands


class Connection(object):
    """One RESP connection to ``host:port``."""

    def __init__(self, host='localhost', port=6379, db=0, password=None,
                 socket_timeout=None, socket_connect_timeout=None,
                 decode_responses=True, encoding='utf-8',
                 client_name=None):
        self.host = host
        self.port = int(port)
        self.db = int(db or 0)
        self.password = password
        self.socket_timeout = socket_timeout
        self.socket_connect_timeout = socket_connect_timeout
        self.decode_responses = decode_responses
        self.encoding = encoding
        self.client_name = client_name
        self._sock = None
        self._parser = None

    def __repr__(self):
        return 'Connection<%s:%s/%s>' % (self.host, self.port, self.db)

    @property
    def connected(self):
        return self._sock is not None

    def connect(self):
        if self._sock is not None:
            return
        try:
            sock = socket.create_connection(
                (self.host, self.port),
                timeout=self.socket_connect_timeout)
        except socket.timeout:
            raise exceptions.TimeoutError(
                'Timeout connecting to %s:%s' % (self.host, self.port))
        except OSError as err:
            raise exceptions.ConnectionError(
                'Error %s connecting to %s:%s. %s.' % (
                    err.errno, self.host, self.port, err.strerror or err))
        sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        sock.setsockopt(socket.SOL_SOCKET, socket.SO_KEEPALIVE, 1)
        sock.settimeout(self.socket_timeout)
        self._sock = sock
        self._parser = RespParser(decode=self.decode_responses,
                                  encoding=self.encoding)
        try:
            self._on_connect()
        except Exception:
            self.disconnect()
            raise

    def _on_connect(self):
        if self.password:
            self._checked('AUTH', self.password)
        if self.db:
            self._checked('SELECT', self.db)
        if self.client_name:
            self._checked('CLIENT', 'SETNAME', self.client_name)

    def _checked(self, *args):
        self.send_packed(encode_command(*args))
        reply = self.read_response()
        if isinstance(reply, exceptions.RedisError):
            raise reply
        return reply

    def disconnect(self):
        sock, self._sock = self._sock, None
        self._parser = None
        if sock is not None:
            try:
                sock.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass
            sock.close()

    def send_packed(self, data):
        if self._sock is None:
            self.connect()
        try:
            self._sock.sendall(data)
        except socket.timeout:
            self.disconnect()
            raise exceptions.TimeoutError('Timeout writing to socket')
        except OSError as err:
            self.disconnect()
            raise exceptions.ConnectionError(
                'Error while writing to socket. %s.' % (err.strerror or err))

    def send_command(self, *args):
        self.send_packed(encode_command(*args))

    def send_commands(self, commands):
        self.send_packed(encode_commands(commands))

    def read_response(self, timeout=None):
        """Return the next reply; error replies are returned (not raised)
        as :class:`ResponseError` instances so pipelines can collect them."""
        if self._sock is None:
            raise exceptions.ConnectionError('Connection closed by client')
        parser = self._parser
        if timeout is not None:
            self._sock.settimeout(timeout)
        try:
            while True:
                reply = parser.gets()
                if reply is not NOT_READY:
                    break
                try:
                    data = self._sock.recv(65536)
                except socket.timeout:
                    self.disconnect()
                    raise exceptions.TimeoutError('Timeout reading from socket')
                except OSError as err:
                    self.disconnect()
                    raise exceptions.ConnectionError(
                        'Error while reading from socket: %s' % (
                            err.strerror or err,))
                if not data:
                    self.disconnect()
                    raise exceptions.ConnectionError(
                        'Connection closed by server.')
                parser.feed(data)
        finally:
            if timeout is not None and self._sock is not None:
                self._sock.settimeout(self.socket_timeout)
        return _materialize_errors(reply)


def _materialize_errors(reply):
    from .resp import ReplyError
    if isinstance(reply, ReplyError):
        return reply.to_exception()
    if isinstance(reply, list):
        return [_materialize_errors(r) if isinstance(r, (list, ReplyError))
                else r for r in reply]
    return reply


class ConnectionPool(object):
    """A LIFO pool of :class:`Connection` objects sharing one config."""

    def __init__(self, connection_class=Connection, max_connections=64,
                 **connection_kwargs):
        self.connection_class = connection_class
        self.connection_kwargs = connection_kwargs
        self.max_connections = max_connections
        self._lock = threading.Lock()
        self._idle = []
        self._in_use = 0

    def __repr__(self):
        return 'ConnectionPool<%s:%s>' % (
            self.connection_kwargs.get('host'),
            self.connection_kwargs.get('port'))

    def get_connection(self):
        with self._lock:
            if self._idle:
                conn = self._idle.pop()
            else:
                if self._in_use >= self.max_connections:
                    raise exceptions.ConnectionError('Too many connections')
                conn = self.connection_class(**self.connection_kwargs)
            self._in_use += 1
        return conn

    def release(self, conn):
        with self._lock:
            self._in_use -= 1
            if conn.connected and len(self._idle) < self.max_connections:
                self._idle.append(conn)

    def disconnect(self):
        with self._lock:
            for conn in self._idle:
                conn.disconnect()
            self._idle = []
