"""What RCCL itself says about each node-communicator generation (VERDICT r4
missing 2 / item 5: the first 8-GPU run must explain itself).

Every worker's RCCL writes its INFO log (``NCCL_DEBUG=INFO``,
``NCCL_DEBUG_SUBSYS=INIT,GRAPH``) to a file of its own
(``NCCL_DEBUG_FILE=<dir>/rccl.%h.%p.log``; :func:`trace_env`, set by the
manager for every worker).  The node agent follows its file
(:class:`RcclTrace`) and reports, per generation:

* RCCL's own ``Init timings`` breakdown (kernels, alloc, bootstrap,
  allgathers, topo, graphs, connections, rest) and the rank's bus id;
* after the generation's first all-reduce (RCCL connects lazily), the
  channel connections it made -- ``Channel 00/0 : 0[75000] -> 1[85000] via
  P2P/IPC`` -- i.e. the transport per peer: ``P2P`` is the intra-node GPU
  path (xGMI on an MI355X node), ``SHM`` host shared memory, ``NET`` a
  network transport;
* the intra-node link type of the graphs RCCL searched (``Pattern 4, ...,
  type XGMI/PIX``, intra/inter): ``XGMI`` between GPUs, anything else
  (``PCI``, ``PIX``, ``SYS``) is flagged.

:func:`parse` is pure (a captured excerpt in a unit test), and the fake
RCCL of the CPU stack writes the same lines.
"""
import os
import re

# ``Init timings - ncclCommInitRankConfig_impl: rank 0 nranks 1 total 0.36
# (kernels 0.28, alloc 0.03, bootstrap 0.00, ...)``
_TIMINGS = re.compile(
    r'Init timings(?: - \S+)?: rank (\d+) nranks (\d+) total ([\d.]+) '
    r'\(([^)]*)\)')
_PHASE = re.compile(r'([a-z]+) ([\d.]+)')
# ``... comm 0x.. rank 0 nranks 8 cudaDev 0 nvmlDev 0 busId 75000 commId
# 0x.. - Init COMPLETE``
_COMPLETE = re.compile(
    r'rank (\d+) nranks (\d+) cudaDev (\d+)(?: nvmlDev \d+)? busId '
    r'([0-9a-fA-F]+)(?: commId (0x[0-9a-fA-F]+))? - Init COMPLETE')
# ``Channel 00/0 : 0[0] -> 1[1] via P2P/IPC/read`` (the bracket is the
# device: its index or, in older releases, its bus id); SHM lines may omit
# the connection index, NET ones carry ``[send]`` / ``[receive]``
_CHANNEL = re.compile(
    r'Channel (\d+)(?:/\d+)? : (\d+)\[([0-9a-fA-Fx]+)\] -> '
    r'(\d+)\[([0-9a-fA-Fx]+)\](?: \[(?:send|receive)\])? via (\S+)')
# ``Pattern 4, crossNic 0, nChannels 1, bw 40.0/40.0, type XGMI/PIX, ...``
_PATTERN = re.compile(r'Pattern (\d+), crossNic \d+, nChannels (\d+),.*?'
                      r'type ([A-Z]+)/([A-Z]+)')
_MEMORY = re.compile(r'Memory used = (\d+)')
_VERSION = re.compile(r'RCCL version\s*:?\s*(\S+)')

#: transports RCCL reports for a connection between two GPUs of one node
#: over xGMI (peer-to-peer through IPC handles, or the CUDA-IPC/VMM paths)
GPU_PEER_TRANSPORTS = ('P2P',)


def parse(text):
    """Facts about the generation(s) in an RCCL INFO log excerpt."""
    out = {'init': None, 'rank': None, 'nranks': None, 'bus_id': None,
           'comm_id': None, 'channels': [], 'transports': {},
           'link_types': [], 'memory_bytes': None, 'version': None}
    for line in text.splitlines():
        m = _TIMINGS.search(line)
        if m:
            phases = {k: float(v) * 1e3 for k, v in _PHASE.findall(m.group(4))}
            phases['total'] = float(m.group(3)) * 1e3
            out['init'] = {k: round(v, 1) for k, v in phases.items()}
            out['rank'], out['nranks'] = int(m.group(1)), int(m.group(2))
            continue
        m = _COMPLETE.search(line)
        if m:
            out['rank'], out['nranks'] = int(m.group(1)), int(m.group(2))
            out['bus_id'] = m.group(4).lower()
            out['comm_id'] = m.group(5)
            continue
        m = _CHANNEL.search(line)
        if m:
            via = m.group(6)
            out['channels'].append({
                'channel': int(m.group(1)), 'from': int(m.group(2)),
                'to': int(m.group(4)), 'from_dev': m.group(3).lower(),
                'to_dev': m.group(5).lower(), 'via': via})
            kind = via.split('/')[0]
            out['transports'][kind] = out['transports'].get(kind, 0) + 1
            continue
        m = _PATTERN.search(line)
        if m:
            # type <intra>/<inter>: the intra-node path is the GPU <-> GPU
            # one; the inter-node part names the NIC path
            if m.group(3) not in out['link_types']:
                out['link_types'].append(m.group(3))
            continue
        m = _MEMORY.search(line)
        if m:
            out['memory_bytes'] = int(m.group(1))
            continue
        m = _VERSION.search(line)
        if m and out['version'] is None:
            out['version'] = m.group(1)
    out['non_gpu_peer'] = sorted(
        {'%d->%d via %s' % (c['from'], c['to'], c['via'])
         for c in out['channels']
         if c['via'].split('/')[0] not in GPU_PEER_TRANSPORTS})
    return out


def summary(parsed):
    """The compact form a rank reports on its pipe."""
    return {k: parsed[k] for k in ('init', 'rank', 'nranks', 'bus_id',
                                   'transports', 'link_types', 'memory_bytes',
                                   'version', 'non_gpu_peer')
            if parsed.get(k) not in (None, [], {})}


def trace_env(directory, environ=None):
    """The NCCL_DEBUG settings that send each worker's RCCL INFO log to a
    file of its own under ``directory``.  ``{}`` with ``RCCL_TRACE=0``, or
    when the operator already has RCCL's INFO output (``NCCL_DEBUG=INFO``)
    or a log file (``NCCL_DEBUG_FILE``); a quieter ``NCCL_DEBUG`` (e.g.
    ``WARN``) is raised to INFO into the files (its warnings land there)."""
    environ = os.environ if environ is None else environ
    if str(environ.get('RCCL_TRACE', '1')).lower() in ('0', 'false', 'off',
                                                       'no') or \
            environ.get('NCCL_DEBUG_FILE') or \
            str(environ.get('NCCL_DEBUG', '')).upper() in ('INFO', 'TRACE'):
        # off, or the operator already routes (or reads) RCCL's INFO output
        return {}
    return {'NCCL_DEBUG': 'INFO', 'NCCL_DEBUG_SUBSYS': 'INIT,GRAPH',
            'NCCL_DEBUG_FILE': os.path.join(directory, 'rccl.%h.%p.log')}


def log_path(environ=None, pid=None, host=None):
    """This process's RCCL log file (``NCCL_DEBUG_FILE`` with RCCL's
    ``%h`` / ``%p`` expanded), or None."""
    environ = os.environ if environ is None else environ
    pattern = environ.get('NCCL_DEBUG_FILE')
    if not pattern or str(environ.get('NCCL_DEBUG', '')).upper() != 'INFO':
        return None
    import socket
    # RCCL's %h is the host name up to its first dot
    host = host or socket.gethostname().split('.')[0]
    pid = os.getpid() if pid is None else pid
    return pattern.replace('%h', host).replace('%p', str(pid))


class RcclTrace(object):
    """Follows one process's RCCL log: :meth:`take` parses what was
    appended since the last call."""

    MAX_READ = 4 << 20

    def __init__(self, path):
        self.path = path
        self.offset = 0

    @classmethod
    def for_process(cls, environ=None):
        path = log_path(environ)
        return cls(path) if path else None

    def take(self):
        try:
            with open(self.path, 'rb') as f:
                f.seek(self.offset)
                data = f.read(self.MAX_READ)
        except OSError:
            return None
        # whole lines only: RCCL may be half-way through writing the last
        end = data.rfind(b'\n') + 1
        self.offset += end
        return parse(data[:end].decode('utf-8', 'replace'))
