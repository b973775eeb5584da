"""GPU inventory for the node-local manager -- without initialising HIP.

The manager process must never create a HIP context: it forks worker
processes, and a process that has initialised the GPU must not exec another
program.  Discovery therefore reads the KFD topology in sysfs (the same
source ROCr enumerates from) and falls back to explicit configuration.

For every GPU it records the HIP ordinal a worker should see through
``HIP_VISIBLE_DEVICES``, the PCI address, the NUMA node and the CPUs local
to it, so workers can be pinned next to their GPU (one process per GPU, host
threads on the socket that owns the GPU's PCIe/xGMI root).
"""
import glob
import os

KFD_NODES = '/sys/class/kfd/kfd/topology/nodes'


class GpuSlot(object):
    """One schedulable device slot."""

    __slots__ = ('index', 'visible_id', 'pci', 'numa_node', 'cpus', 'kind',
                 'hbm_bytes', 'cu_count', 'pci_verified')

    def __init__(self, index, visible_id, pci=None, numa_node=-1, cpus=None,
                 kind='gpu', hbm_bytes=0, cu_count=0):
        self.index = index
        self.visible_id = visible_id
        self.pci = pci
        self.numa_node = numa_node
        self.cpus = cpus or []
        self.kind = kind
        self.hbm_bytes = hbm_bytes
        self.cu_count = cu_count
        # a process pinned to it reported the same PCI address through HIP
        self.pci_verified = False

    def to_dict(self):
        return {k: getattr(self, k) for k in self.__slots__}

    def __repr__(self):
        return 'GpuSlot(%d, visible=%s, numa=%s)' % (
            self.index, self.visible_id, self.numa_node)


def _read_properties(path):
    props = {}
    try:
        with open(path) as handle:
            for line in handle:
                parts = line.split()
                if len(parts) == 2:
                    try:
                        props[parts[0]] = int(parts[1])
                    except ValueError:
                        pass
    except OSError:
        pass
    return props


def parse_cpulist(text):
    cpus = []
    for part in text.strip().split(','):
        if not part:
            continue
        if '-' in part:
            lo, hi = part.split('-')
            cpus.extend(range(int(lo), int(hi) + 1))
        else:
            cpus.append(int(part))
    return cpus


def _pci_address(props):
    loc = props.get('location_id')
    if loc is None:
        return None
    domain = props.get('domain', 0)
    return '%04x:%02x:%02x.%d' % (domain, (loc >> 8) & 0xff, (loc >> 3) & 0x1f,
                                  loc & 0x7)


def normalize_pci(text):
    """Canonical ``dddd:bb:dd.f`` (lower case) of a PCI address as KFD,
    amdsmi or ``hipDeviceGetPCIBusId`` print it, or ``None``."""
    if not text:
        return None
    try:
        head, func = str(text).strip().lower().rsplit('.', 1)
        parts = head.split(':')
        if len(parts) == 2:
            parts = ['0'] + parts
        domain, bus, dev = (int(p, 16) for p in parts)
        return '%04x:%02x:%02x.%d' % (domain, bus, dev, int(func, 16))
    except (ValueError, TypeError):
        return None


def local_cpus(pci):
    """``(numa node, [cpus])`` local to a PCI device (sysfs)."""
    return _local_cpus(pci)


def _local_cpus(pci):
    if not pci:
        return -1, []
    base = '/sys/bus/pci/devices/%s' % pci
    numa = -1
    try:
        with open(base + '/numa_node') as handle:
            numa = int(handle.read().strip())
    except (OSError, ValueError):
        pass
    try:
        with open(base + '/local_cpulist') as handle:
            return numa, parse_cpulist(handle.read())
    except OSError:
        return numa, []


def kfd_gpus(root=KFD_NODES):
    """GPU nodes from the KFD topology, in HIP enumeration order."""
    found = []
    for node in sorted(glob.glob(os.path.join(root, '*')),
                       key=lambda p: int(os.path.basename(p))
                       if os.path.basename(p).isdigit() else 1 << 30):
        props = _read_properties(os.path.join(node, 'properties'))
        if not props.get('gpu_id') or not props.get('simd_count'):
            continue  # CPU node
        pci = _pci_address(props)
        numa, cpus = _local_cpus(pci)
        simds = props.get('simd_count', 0)
        per_cu = props.get('simd_per_cu', 4) or 4
        found.append({'pci': pci, 'numa_node': numa, 'cpus': cpus,
                      'cu_count': simds // per_cu})
    return found


def amdsmi_gpus():
    """Fallback inventory through amdsmi (no HIP init) when the KFD
    topology is not readable (e.g. inside some containers)."""
    try:
        import amdsmi
        amdsmi.amdsmi_init()
    except Exception:  # pylint: disable=broad-except
        return []
    found = []
    try:
        for handle in amdsmi.amdsmi_get_processor_handles():
            info = {'pci': None, 'numa_node': -1, 'cpus': [], 'cu_count': 0}
            try:
                info['pci'] = amdsmi.amdsmi_get_gpu_device_bdf(handle)
                numa, cpus = _local_cpus(info['pci'])
                info['cpus'] = cpus
                info['numa_node'] = numa
            except Exception:  # pylint: disable=broad-except
                pass
            try:
                info['numa_node'] = int(
                    amdsmi.amdsmi_topo_get_numa_node_number(handle))
            except Exception:  # pylint: disable=broad-except
                pass
            found.append(info)
    finally:
        try:
            amdsmi.amdsmi_shut_down()
        except Exception:  # pylint: disable=broad-except
            pass
    return found


def _visible_filter(env):
    for name in ('HIP_VISIBLE_DEVICES', 'ROCR_VISIBLE_DEVICES',
                 'CUDA_VISIBLE_DEVICES'):
        value = env.get(name)
        if value:
            return [v.strip() for v in value.split(',') if v.strip()]
    return None


def discover(gpu_ids='', env=None, cpu_slots=0, kfd_root=KFD_NODES):
    """Return the list of :class:`GpuSlot` this manager may schedule on.

    Args:
        gpu_ids: ``GPU_IDS`` setting, e.g. ``'0,1,2,3'``; '' = all visible.
        env: environment (defaults to ``os.environ``).
        cpu_slots: when no GPU exists, create this many ``kind='cpu'``
            virtual slots (mock-worker plumbing runs, BASELINE config 1).
    """
    env = os.environ if env is None else env
    nodes = kfd_gpus(kfd_root) or amdsmi_gpus()
    visible = _visible_filter(env)
    if visible is not None:
        physical = [int(v) for v in visible if v.isdigit()]
    else:
        physical = list(range(len(nodes)))
    if gpu_ids:
        wanted = [int(g) for g in str(gpu_ids).split(',') if g.strip()]
        # GPU_IDS index the visible list
        physical = [physical[i] for i in wanted if i < len(physical)] \
            if nodes else wanted
    slots = []
    for index, phys in enumerate(physical):
        info = nodes[phys] if phys < len(nodes) else {}
        slots.append(GpuSlot(index=index, visible_id=str(phys),
                             pci=info.get('pci'),
                             numa_node=info.get('numa_node', -1),
                             cpus=info.get('cpus', []),
                             cu_count=info.get('cu_count', 0)))
    if not slots and cpu_slots:
        slots = [GpuSlot(index=i, visible_id='', kind='cpu')
                 for i in range(cpu_slots)]
    return slots
