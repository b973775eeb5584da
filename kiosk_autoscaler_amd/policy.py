"""Scaling decision functions (components C11, C12 and the sum in C14).

Pure functions of (queue key counts, bounds, current replicas) so they can be
tested exhaustively and shared by the live autoscaler, the simulator in
:mod:`kiosk_autoscaler_amd.bench.sim` and the benchmark.

``reference`` reproduces the reference's arithmetic *exactly*, quirks
included (SURVEY §3.2 truth table):

* per-queue ``keys // keys_per_pod`` (floor: fewer than ``KEYS_PER_POD``
  keys never scale up from zero; ``autoscaler/autoscaler.py:217``);
* each per-queue value is clipped with the *global* ``current``, then the
  sum is clipped again (``autoscaler.py:254-260``) -- so two queues with
  one key each can hold 2x ``current`` and ``MIN_PODS`` counts per queue;
* ``0 < desired < current`` holds ``current`` (``autoscaler.py:207-208``):
  scale-down only to exactly zero.

``strict`` is the opt-in fix (SURVEY §3.2 "Recommendation"): global sum,
ceiling division, scale-down allowed to ``max(min_pods, busy)``.
"""


def clip_pod_count(desired_pods, min_pods, max_pods, current_pods):
    """Clamp to [min, max]; then never shrink a live set while work exists."""
    if desired_pods > max_pods:
        desired_pods = max_pods
    elif desired_pods < min_pods:
        desired_pods = min_pods
    if 0 < desired_pods < current_pods:
        desired_pods = current_pods
    return desired_pods


def desired_for_queue(keys, keys_per_pod, min_pods, max_pods, current_pods):
    """Per-queue demand: floor(keys / keys_per_pod), then :func:`clip_pod_count`."""
    return clip_pod_count(keys // keys_per_pod, min_pods, max_pods,
                          current_pods)


def decide_reference(keys_by_queue, min_pods, max_pods, keys_per_pod,
                     current_pods, busy=0):
    """Bit-compatible reference decision (``Autoscaler.scale``)."""
    del busy  # the reference does not know which pods are busy
    total = 0
    for keys in keys_by_queue.values():
        total += desired_for_queue(keys, keys_per_pod, min_pods, max_pods,
                                   current_pods)
    return clip_pod_count(total, min_pods, max_pods, current_pods)


def decide_strict(keys_by_queue, min_pods, max_pods, keys_per_pod,
                  current_pods, busy=0):
    """Global-sum, ceil-division policy that may shrink to the busy floor.

    ``busy`` is the number of workers currently holding a key: they are
    never reclaimed, so the target never drops below it."""
    del current_pods
    total = sum(keys_by_queue.values())
    desired = -(-total // keys_per_pod) if total > 0 else 0
    desired = max(min_pods, min(max_pods, desired))
    return max(desired, min(busy, max_pods))


POLICIES = {
    'reference': decide_reference,
    'strict': decide_strict,
}


def decide(keys_by_queue, min_pods, max_pods, keys_per_pod, current_pods,
           policy='reference', busy=0):
    """Dispatch to a named policy; raises ``ValueError`` on unknown names."""
    try:
        func = POLICIES[policy]
    except KeyError:
        raise ValueError('unknown SCALE_POLICY %r (choose from %s)' % (
            policy, sorted(POLICIES)))
    if keys_per_pod <= 0:
        raise ValueError('KEYS_PER_POD must be positive, got %r' % keys_per_pod)
    return func(keys_by_queue, min_pods, max_pods, keys_per_pod,
                current_pods, busy=busy)
