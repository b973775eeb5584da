"""Assignment parsing and process pinning for the worker: stdlib only, so
a cold-spawned worker can pin itself (``HIP_VISIBLE_DEVICES``, CPU affinity)
and start opening the device before the heavier runtime modules load."""
import json
import os


def parse_assignment(text):
    return json.loads(text) if isinstance(text, str) else text


def apply_assignment_env(assignment, env=None):
    """Put the template env and the GPU pin into ``os.environ``.

    Must run before anything initialises HIP: the runtime reads
    ``HIP_VISIBLE_DEVICES`` once, at init."""
    env = os.environ if env is None else env
    template = assignment.get('template', {})
    for key, value in template.get('env', {}).items():
        env[key] = str(value)
    gpu = assignment.get('gpu')
    if gpu not in (None, ''):
        # `gpu` is an ordinal of the full device list.  If the node filters
        # at the ROCr level, re-filter there (HIP would renumber from 0).
        env.pop('CUDA_VISIBLE_DEVICES', None)
        visible = [str(v) for v in assignment.get('visible') or ()]
        if visible and str(gpu) in visible:
            # WORKER_PIN=visible: every managed GPU stays visible (RCCL
            # sees its peers as devices of this process) and the worker's
            # own is selected in-process: KIOSK_DEVICE is its ordinal in
            # that list, which HIP numbers from 0
            listed = ','.join(visible)
            ordinal = visible.index(str(gpu))
        else:
            listed, ordinal = str(gpu), 0
        if env.get('ROCR_VISIBLE_DEVICES'):
            env['ROCR_VISIBLE_DEVICES'] = listed
            env.pop('HIP_VISIBLE_DEVICES', None)
        else:
            env['HIP_VISIBLE_DEVICES'] = listed
        if ordinal or visible:
            env['KIOSK_DEVICE'] = str(ordinal)
        else:
            env.pop('KIOSK_DEVICE', None)
    cpus = assignment.get('cpus') or []
    if cpus and hasattr(os, 'sched_setaffinity'):
        try:
            os.sched_setaffinity(0, set(int(c) for c in cpus))
        except OSError:
            pass
    return env


def device_ordinal(env=None):
    """The HIP ordinal of this worker's GPU inside its process: 0 when it
    is the only visible device (``WORKER_PIN=isolate``), its position in
    the managed list with ``WORKER_PIN=visible`` (``KIOSK_DEVICE``)."""
    env = os.environ if env is None else env
    try:
        return int(env.get('KIOSK_DEVICE') or 0)
    except ValueError:
        return 0
