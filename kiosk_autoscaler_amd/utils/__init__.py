"""Observability and host-side helpers (events, logging, HBM sizing, roctx)."""
from .events import EventLog, NULL as NULL_EVENTS, now_ns
from .logs import LOG_FORMAT, initialize_logger
from .trace import trace_range, mark as trace_mark

__all__ = ['EventLog', 'NULL_EVENTS', 'now_ns', 'LOG_FORMAT',
           'initialize_logger', 'trace_range', 'trace_mark']
