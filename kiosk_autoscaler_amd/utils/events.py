"""Structured, timestamped lifecycle events.

Every stage on the scale-up critical path emits one event:
``key_enqueued``, ``tick``, ``scale``, ``worker_spawn``, ``worker_assigned``,
``hip_ready``, ``weights_ready``, ``warmstart_done``, ``worker_ready``,
``fence_done``, ``key_start``, ``key_done``, ``worker_exit`` ...

Timestamps are ``CLOCK_MONOTONIC`` nanoseconds, which is system-wide on
Linux, so events from the manager, the workers and the load generator are
directly comparable.  Sinks: a JSONL file (``EVENT_LOG``) and/or a Redis list
(``kiosk:events``) so the benchmark can collect events from every process.
"""
import json
import os
import threading
import time

EVENTS_KEY = 'kiosk:events'


def now_ns():
    return time.monotonic_ns()


class EventLog(object):
    """Thread-safe event sink.  ``emit(kind, **fields)``."""

    def __init__(self, path=None, redis_client=None, redis_key=EVENTS_KEY,
                 source=None):
        self.path = path or None
        self.redis_client = redis_client
        self.redis_key = redis_key
        self.source = source or 'pid%d' % os.getpid()
        self._lock = threading.Lock()
        self._send_lock = threading.Lock()   # one socket, many threads
        self._fh = None
        self.records = []
        self.keep = False
        # in-process consumers of every record (e.g. the Prometheus
        # exporter); an observer's failure never reaches the emitter
        self.observers = []

    def emit(self, _event, t_ns=None, **fields):
        record = {"ev": _event, 't': now_ns() if t_ns is None else int(t_ns),
                  'src': self.source}
        record.update(fields)
        line = json.dumps(record, sort_keys=True, default=str)
        with self._lock:
            if self.keep:
                self.records.append(record)
            if self.path:
                if self._fh is None:
                    self._fh = open(self.path, 'a', buffering=1)
                self._fh.write(line + '\n')
        if self.redis_client is not None:
            try:
                with self._send_lock:
                    self.redis_client.rpush(self.redis_key, line)
            except Exception:  # pylint: disable=broad-except
                pass  # observability must never take the control loop down
        for observer in list(self.observers):
            try:
                observer(record)
            except Exception:  # pylint: disable=broad-except
                pass
        return record

    def close(self):
        with self._lock:
            if self._fh is not None:
                self._fh.close()
                self._fh = None


class _NullLog(object):
    records = ()

    def emit(self, _event, t_ns=None, **fields):
        return None

    def close(self):
        pass


NULL = _NullLog()


def read_jsonl(path):
    records = []
    if not path or not os.path.exists(path):
        return records
    with open(path) as handle:
        for line in handle:
            line = line.strip()
            if line:
                records.append(json.loads(line))
    return records


def drain_redis(redis_client, key=EVENTS_KEY):
    """Pop every event currently stored in Redis (oldest first)."""
    out = []
    pipe = redis_client.pipeline(transaction=True)
    pipe.lrange(key, 0, -1)
    pipe.delete(key)
    lines, _ = pipe.execute()
    for line in lines or []:
        out.append(json.loads(line))
    return out
