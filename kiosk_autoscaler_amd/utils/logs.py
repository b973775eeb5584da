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

A process that dies mid-tick (SIGKILL, a segfault, the OOM killer) cannot
flush, and the records it held are exactly the ones that explain the death.
So each held record is also copied, unformatted, into a memory-mapped
journal beside the log file (``<log>.pending``, :class:`_Journal`): a copy
into the page cache, no system call, and the kernel keeps those pages when
the process dies.  A flush empties the journal.  The next process that sets
up logging on that file writes what a dead predecessor left there first,
under a WARNING that says so.
"""
import atexit
import collections
import logging
import logging.handlers
import mmap
import os
import struct
import sys

LOG_FORMAT = '[%(asctime)s]:[%(levelname)s]:[%(name)s]: %(message)s'


class _Journal:
    """The held records' crash copy: a fixed-size memory-mapped file.
    Layout: 8-byte magic, the used length (u64), then one entry per record,
    ``created<TAB>levelno<TAB>name<TAB>message<NUL>``.  The length is
    written after the entry, so a death between the two loses that one
    entry, never the ones before it."""

    MAGIC = b'kioskjr1'
    HEAD = 16

    def __init__(self, path, size=1 << 20):
        self.path = path
        fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o644)
        try:
            if os.fstat(fd).st_size != size:
                os.ftruncate(fd, size)
            self._map = mmap.mmap(fd, size)
        finally:
            os.close(fd)
        self.size = size
        if self._map[:8] != self.MAGIC:
            self._map[:8] = self.MAGIC
            self._set_used(self.HEAD)
        self.used = self._get_used()

    def _get_used(self):
        used = struct.unpack_from('<Q', self._map, 8)[0]
        return used if self.HEAD <= used <= self.size else self.HEAD

    def _set_used(self, used):
        struct.pack_into('<Q', self._map, 8, used)
        self.used = used

    def leftover(self):
        """Records a process that died with them held left here."""
        out = []
        body = bytes(self._map[self.HEAD:self._get_used()])
        for entry in body.split(b'\0'):
            parts = entry.decode('utf-8', 'replace').split('\t', 3)
            if len(parts) != 4:
                continue
            try:
                created, levelno = float(parts[0]), int(parts[1])
            except ValueError:
                continue
            out.append(logging.makeLogRecord({
                'name': parts[2], 'levelno': levelno,
                'levelname': logging.getLevelName(levelno),
                'msg': parts[3], 'created': created,
                'msecs': (created - int(created)) * 1000}))
        return out

    def append(self, record):
        """False when the journal is full (the caller drains first)."""
        data = ('%r\t%d\t%s\t%s\0' % (record.created, record.levelno,
                                        record.name, record.msg)).encode(
            'utf-8', 'replace')
        # the length in the file, not a cached one: two handlers of one
        # process may share the journal
        used = self._get_used()
        end = used + len(data)
        if end > self.size:
            return False
        self._map[used:end] = data
        self._set_used(end)
        return True

    def clear(self):
        if self._get_used() != self.HEAD:
            self._set_used(self.HEAD)

    def close(self):
        try:
            self._map.close()
        except (ValueError, OSError):
            pass


class DeferredHandler(logging.Handler):
    """Keeps records (message text fixed at the call) until :meth:`flush`,
    then hands them to ``handlers``, each at its own level.  WARNING and
    above flush at once; so does a full buffer and interpreter exit.  With
    ``journal`` (a path) the held records survive the process's death
    (:class:`_Journal`); records a dead predecessor left there are written
    first."""

    CAPACITY = 4096

    def __init__(self, handlers, journal=None):
        super().__init__(logging.DEBUG)
        self.handlers = list(handlers)
        self._records = collections.deque()
        self._journal = None
        if journal:
            try:
                self._journal = _Journal(journal)
            except (OSError, ValueError):
                self._journal = None
        if self._journal is not None:
            self._recover()
        atexit.register(self.close)

    def _recover(self):
        records = self._journal.leftover()
        if not records:
            return
        note = logging.makeLogRecord({
            'name': __name__, 'levelno': logging.WARNING,
            'levelname': 'WARNING',
            'msg': 'Recovered %d log records that a previous process held '
                   'when it died (%s).' % (len(records), self._journal.path)})
        self._records.extend([note] + records)
        self._drain()

    def emit(self, record):
        # the text as it reads now (its arguments may change later)
        record.msg = record.getMessage()
        record.args = None
        journal = self._journal
        if journal is not None and record.levelno < logging.WARNING and \
                not journal.append(record):
            self._drain()
            journal.append(record)
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
        if self._journal is not None:
            self._journal.clear()

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
        if self._journal is not None:
            self._journal.close()
            self._journal = None
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
        root.addHandler(DeferredHandler(
            handlers, journal=log_file + '.pending' if log_file else None))
    else:
        for handler in handlers:
            root.addHandler(handler)

    logging.getLogger('GpuManagerTransport').setLevel(logging.INFO)
    return root
