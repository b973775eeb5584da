"""The in-flight key convention shared by the tally, the workers and the
manager's requeue (``processing-<queue>:<worker-id>[.<slot>]``).

The reference counts ``processing-<q>:*`` keys (``autoscaler/
autoscaler.py:69-71``); a batched worker here holds one key per batch slot,
slot 0 without a suffix and slot ``i > 0`` as ``.<i>``.  Worker ids may
contain dots themselves (resource names are DNS-1123 subdomains, e.g.
``my.app``), so only a trailing ``.<digits>`` is the slot.
"""
import re

_SLOT = re.compile(r'\.\d+$')


def processing_key(queue, worker_id, slot=0):
    suffix = '' if not slot else '.%d' % slot
    return 'processing-%s:%s%s' % (queue, worker_id, suffix)


def worker_of(key):
    """The worker id of a processing key (``None`` if it has no ``:``)."""
    if ':' not in key:
        return None
    return _SLOT.sub('', key.split(':', 1)[1])
