"""Exception hierarchy of the in-tree Redis client.

Mirrors the error classes the reference's retry logic branches on
(``redis.exceptions.ConnectionError`` / ``ResponseError``;
reference ``autoscaler/redis.py:177-200``) so the retry semantics can be kept
without redis-py, which is not available in this environment.
"""


class RedisError(Exception):
    """Base class of every error raised by :mod:`kiosk_autoscaler_amd.redisq`."""


class ConnectionError(RedisError):  # pylint: disable=redefined-builtin
    """The TCP connection could not be made, was reset, or timed out."""


class TimeoutError(ConnectionError):  # pylint: disable=redefined-builtin
    """A socket operation exceeded its timeout."""


class ResponseError(RedisError):
    """The server answered a command with a RESP error (``-ERR ...``)."""


class BusyLoadingError(ConnectionError):
    """The server is loading its dataset and cannot serve yet."""


class DataError(RedisError):
    """A command argument could not be encoded."""


class ProtocolError(ConnectionError):
    """The byte stream from the server is not valid RESP."""


def parse_error(message):
    """Map a server error string to the most specific exception class."""
    if message.startswith('LOADING'):
        return BusyLoadingError(message)
    return ResponseError(message)
