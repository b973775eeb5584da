"""RESP2 wire codec: command encoding and an incremental reply parser.

The reference talks to Redis through redis-py (``autoscaler/redis.py:158-161``).
redis-py is not installable here, so the framework carries its own codec.
The parser is incremental (feed bytes, pop complete replies) so one code
path serves blocking sockets, pipelines and the in-tree test server.
"""
from .exceptions import DataError, ProtocolError, parse_error

CRLF = b'\r\n'


def _to_bytes(value):
    if isinstance(value, bytes):
        return value
    if isinstance(value, str):
        return value.encode('utf-8')
    if isinstance(value, bool):
        # redis-py refuses bools because their meaning is ambiguous.
        raise DataError('Invalid input of type bool; convert to int or str')
    if isinstance(value, (int, float)):
        return repr(value).encode('ascii')
    if isinstance(value, memoryview):
        return value.tobytes()
    raise DataError('Invalid input of type %s' % type(value).__name__)


def encode_command(*args):
    """Encode one command as a RESP array of bulk strings."""
    parts = [b'*%d\r\n' % len(args)]
    for arg in args:
        data = _to_bytes(arg)
        parts.append(b'$%d\r\n' % len(data))
        parts.append(data)
        parts.append(CRLF)
    return b''.join(parts)


def encode_commands(commands):
    """Encode several commands back to back (pipelining)."""
    return b''.join(encode_command(*cmd) for cmd in commands)


class ReplyError(object):
    """A RESP error reply held as a value (used inside arrays / pipelines)."""

    __slots__ = ('message',)

    def __init__(self, message):
        self.message = message

    def to_exception(self):
        return parse_error(self.message)

    def __repr__(self):
        return 'ReplyError(%r)' % self.message

    def __eq__(self, other):
        return isinstance(other, ReplyError) and other.message == self.message


_INCOMPLETE = object()


class RespParser(object):
    """Incremental RESP2 parser.

    ``feed(data)`` appends bytes; ``gets()`` returns the next complete reply
    or the module-level sentinel ``NOT_READY``.  Error replies come back as
    :class:`ReplyError` values so callers decide whether to raise.
    """

    def __init__(self, decode=True, encoding='utf-8'):
        self._buf = bytearray()
        self._pos = 0
        self.decode = decode
        self.encoding = encoding

    def feed(self, data):
        if self._pos and self._pos > 65536:
            del self._buf[:self._pos]
            self._pos = 0
        self._buf.extend(data)

    def pending(self):
        return len(self._buf) - self._pos

    def gets(self):
        start = self._pos
        result = self._parse()
        if result is _INCOMPLETE:
            self._pos = start
            return NOT_READY
        return result

    def _readline(self):
        end = self._buf.find(CRLF, self._pos)
        if end < 0:
            return None
        line = bytes(self._buf[self._pos:end])
        self._pos = end + 2
        return line

    def _parse(self):
        line = self._readline()
        if line is None:
            return _INCOMPLETE
        if not line:
            raise ProtocolError('empty RESP line')
        kind, rest = line[:1], line[1:]
        if kind == b'+':
            return rest.decode(self.encoding) if self.decode else rest
        if kind == b'-':
            return ReplyError(rest.decode(self.encoding, 'replace'))
        if kind == b':':
            try:
                return int(rest)
            except ValueError:
                raise ProtocolError('bad integer reply %r' % rest)
        if kind == b'$':
            length = int(rest)
            if length < 0:
                return None
            end = self._pos + length
            if len(self._buf) < end + 2:
                return _INCOMPLETE
            data = bytes(self._buf[self._pos:end])
            self._pos = end + 2
            if self.decode:
                try:
                    return data.decode(self.encoding)
                except UnicodeDecodeError:
                    return data
            return data
        if kind == b'*':
            count = int(rest)
            if count < 0:
                return None
            items = []
            for _ in range(count):
                item = self._parse()
                if item is _INCOMPLETE:
                    return _INCOMPLETE
                items.append(item)
            return items
        raise ProtocolError('unknown RESP type byte %r' % kind)


class _NotReady(object):
    def __repr__(self):
        return 'NOT_READY'

    def __bool__(self):
        return False


NOT_READY = _NotReady()


# ---------------------------------------------------------------------------
# Server-side encoders (used by the in-tree Python RESP server).
# ---------------------------------------------------------------------------

class SimpleString(str):
    """Marks a reply that must go out as ``+OK``-style simple string."""


def encode_reply(value):
    """Encode a Python value as a RESP2 reply (server direction)."""
    if value is None:
        return b'$-1\r\n'
    if isinstance(value, ReplyError):
        return b'-' + value.message.encode('utf-8') + CRLF
    if isinstance(value, SimpleString):
        return b'+' + value.encode('utf-8') + CRLF
    if isinstance(value, bool):
        return b':%d\r\n' % int(value)
    if isinstance(value, int):
        return b':%d\r\n' % value
    if isinstance(value, (bytes, bytearray, str)):
        data = _to_bytes(bytes(value) if isinstance(value, bytearray) else value)
        return b'$%d\r\n%s\r\n' % (len(data), data)
    if isinstance(value, float):
        data = repr(value).encode('ascii')
        return b'$%d\r\n%s\r\n' % (len(data), data)
    if isinstance(value, (list, tuple)):
        return b'*%d\r\n' % len(value) + b''.join(encode_reply(v) for v in value)
    if isinstance(value, NullArray):
        return b'*-1\r\n'
    raise DataError('cannot encode reply of type %s' % type(value).__name__)


class NullArray(object):
    """The RESP2 null multi-bulk (``*-1``), e.g. a timed-out BLPOP."""


NULL_ARRAY = NullArray()
