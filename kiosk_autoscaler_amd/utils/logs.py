"""Logging setup (component C16).

Same formatter string, root level and rotating file policy as the reference
(``scale.py:42-66``) so log diffs stay comparable: DEBUG root, stdout at
DEBUG (``debug_mode``) or INFO, ``autoscaler.log`` rotating at 10 MB x 10
backups at DEBUG.  The reference pins ``kubernetes.client.rest`` at INFO; the
equivalent chatty logger here is the GPU-manager transport.
"""
import logging
import logging.handlers
import sys

LOG_FORMAT = '[%(asctime)s]:[%(levelname)s]:[%(name)s]: %(message)s'


def initialize_logger(debug_mode=True, log_file='autoscaler.log',
                      max_bytes=10000000, backup_count=10, stream=None):
    root = logging.getLogger()
    root.setLevel(logging.DEBUG)
    formatter = logging.Formatter(LOG_FORMAT)

    console = logging.StreamHandler(stream=stream or sys.stdout)
    console.setFormatter(formatter)
    console.setLevel(logging.DEBUG if debug_mode else logging.INFO)
    root.addHandler(console)

    if log_file:
        handler = logging.handlers.RotatingFileHandler(
            filename=log_file, maxBytes=max_bytes, backupCount=backup_count)
        handler.setFormatter(formatter)
        handler.setLevel(logging.DEBUG)
        root.addHandler(handler)

    logging.getLogger('GpuManagerTransport').setLevel(logging.INFO)
    return root
