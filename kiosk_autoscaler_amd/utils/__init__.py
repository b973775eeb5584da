"""Observability and host-side helpers (events, logging, HBM sizing, roctx)."""
from .events import EventLog, NULL as NULL_EVENTS, now_ns
from .logs import LOG_FORMAT, initialize_logger

__all__ = ['EventLog', 'NULL_EVENTS', 'now_ns', 'LOG_FORMAT',
           'initialize_logger']
