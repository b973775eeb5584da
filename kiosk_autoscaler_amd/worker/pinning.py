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
        if env.get('ROCR_VISIBLE_DEVICES'):
            env['ROCR_VISIBLE_DEVICES'] = str(gpu)
            env.pop('HIP_VISIBLE_DEVICES', None)
        else:
            env['HIP_VISIBLE_DEVICES'] = str(gpu)
    cpus = assignment.get('cpus') or []
    if cpus and hasattr(os, 'sched_setaffinity'):
        try:
            os.sched_setaffinity(0, set(int(c) for c in cpus))
        except OSError:
            pass
    return env
