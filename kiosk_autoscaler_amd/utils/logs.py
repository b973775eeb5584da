"""Logging setup (component C16).

Same formatter string, root level and rotating file policy as the reference
(``scale.py:42-66``) so log diffs stay comparable: DEBUG root, stdout at
DEBUG (``debug_mode``) or INFO, ``autoscaler.log`` rotating at 10 MB x 10
backups at DEBUG.  The reference pins ``kubernetes.client.rest`` at INFO; the
equivalent chatty logger here is the GPU-manager transport.

The records are formatted and written after the tick, not while it runs
(:class:`DeferredHandler`, flushed by ``cli.run_loop`` after every tick,
at once for WARNING and above): the reconcile tick emits ~8 DEBUG records,
and written inline -- two handlers, a write per record each, the rotating
file's seek -- they took it from 0.12 to 0.75 ms, on the first-key latency
path, since the scale-up decision waits for the tick (``profiles/r5_boot/``).
Same records, same format, same files.
"""
import atexit
import collections
import logging
import logging.handlers
import sys

LOG_FORMAT = '[%(asctime)s]:[%(levelname)s]:[%(name)s]: %(message)s'


class DeferredHandler(logging.Handler):
    """Keeps records (message text fixed at the call) until :meth:`flush`,
    then hands them to ``handlers``, each at its own level.  WARNING and
    above flush at once; so does a full buffer and interpreter exit."""

    CAPACITY = 4096

    def __init__(self, handlers):
        super().__init__(logging.DEBUG)
        self.handlers = list(handlers)
        self._records = collections.deque()
        atexit.register(self.close)

    def emit(self, record):
        # the text as it reads now (its arguments may change later)
        record.msg = record.getMessage()
        record.args = None
        self._records.append(record)
        if record.levelno >= logging.WARNING or \
                len(self._records) >= self.CAPACITY:
            self._drain()

    def _drain(self):
        while self._records:
            record = self._records.popleft()
            for handler in self.handlers:
                if record.levelno >= handler.level:
                    handler.handle(record)
        for handler in self.handlers:
            handler.flush()

    def flush(self):
        self.acquire()
        try:
            self._drain()
        finally:
            self.release()

    def close(self):
        self.flush()
        for handler in self.handlers:
            handler.close()
        self.handlers = []
        super().close()


def flush_deferred(logger=None):
    """Write what the deferred handlers of ``logger`` (root) hold."""
    for handler in (logger or logging.getLogger()).handlers:
        if isinstance(handler, DeferredHandler):
            handler.flush()


def initialize_logger(debug_mode=True, log_file='autoscaler.log',
                      max_bytes=10000000, backup_count=10, stream=None,
                      deferred=True):
    root = logging.getLogger()
    root.setLevel(logging.DEBUG)
    formatter = logging.Formatter(LOG_FORMAT)
    handlers = []

    console = logging.StreamHandler(stream=stream or sys.stdout)
    console.setFormatter(formatter)
    console.setLevel(logging.DEBUG if debug_mode else logging.INFO)
    handlers.append(console)

    if log_file:
        handler = logging.handlers.RotatingFileHandler(
            filename=log_file, maxBytes=max_bytes, backupCount=backup_count)
        handler.setFormatter(formatter)
        handler.setLevel(logging.DEBUG)
        handlers.append(handler)

    if deferred:
        root.addHandler(DeferredHandler(handlers))
    else:
        for handler in handlers:
            root.addHandler(handler)

    logging.getLogger('GpuManagerTransport').setLevel(logging.INFO)
    return root
