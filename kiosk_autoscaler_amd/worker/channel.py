"""Worker side of the manager <-> worker pipe protocol.

Manager -> worker (``--cmd-fd``), one JSON object per line:
``assign`` (GPU, template, ids), ``drain`` / ``undrain``, ``fence`` /
``fence_abort``, ``exit``.  Worker -> manager (``--ev-fd``): ``standby``, ``stage``,
``ready``, ``busy`` / ``beat`` / ``idle``, ``fenced``, ``recycled``,
``error``.
"""
import json
import os
import queue
import select
import threading
import time

#: ``read_command(timeout=...)`` result when nothing arrived in time
TIMEOUT = {'cmd': '__timeout__'}


class Channel(object):
    def __init__(self, cmd_fd=None, ev_fd=None):
        self.cmd_fd = cmd_fd
        self.ev_fd = ev_fd
        self._lock = threading.Lock()
        self._buf = b''
        self.commands = queue.Queue()
        # cmd -> callable run on the reader thread instead of queueing: fence
        # commands must reach the fence agent while the main thread is
        # inside a key (it only drains ``commands`` between keys)
        self.direct = {}
        self._reader = None

    def emit(self, ev, **fields):
        if self.ev_fd is None:
            return
        fields['ev'] = ev
        fields.setdefault('t', time.monotonic_ns())
        data = (json.dumps(fields, default=str) + '\n').encode()
        with self._lock:
            try:
                os.write(self.ev_fd, data)
            except OSError:
                pass

    def _read_line(self):
        while b'\n' not in self._buf:
            try:
                chunk = os.read(self.cmd_fd, 65536)
            except OSError:
                chunk = b''
            if not chunk:
                return None
            self._buf += chunk
        line, self._buf = self._buf.split(b'\n', 1)
        return json.loads(line)

    def read_command(self, timeout=None):
        """Blocking read of the next command (``None`` on EOF; after
        ``timeout`` seconds without one, :data:`TIMEOUT`).  Once the reader
        thread runs (after the first assignment), commands come from its
        queue."""
        if self.cmd_fd is None:
            return None
        if self._reader is not None:
            try:
                message = self.commands.get(timeout=timeout)
            except queue.Empty:
                return TIMEOUT
            return None if message.get('cmd') == 'eof' else message
        if timeout is not None and b'\n' not in self._buf:
            ready, _, _ = select.select([self.cmd_fd], [], [], timeout)
            if not ready:
                return TIMEOUT
        return self._read_line()

    def start_reader(self):
        """Forward commands to :attr:`commands` from a daemon thread."""
        if self.cmd_fd is None or self._reader is not None:
            return

        def pump():
            while True:
                message = self._read_line()
                handler = (self.direct.get(message.get('cmd'))
                           if message is not None else None)
                if handler is not None:
                    handler(message)
                    continue
                self.commands.put(message if message is not None
                                  else {'cmd': 'eof'})
                if message is None:
                    return
        self._reader = threading.Thread(target=pump, name='worker-cmd',
                                        daemon=True)
        self._reader.start()
