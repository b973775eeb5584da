"""Decision semantics: the characterised golden truth table."""
import itertools

import pytest

from kiosk_autoscaler_amd import policy


@pytest.mark.parametrize('args,expected', [
    ((0, 0, 1, 1), 0),   # scale to zero allowed
    ((5, 0, 1, 0), 1),   # max clamp
    ((2, 0, 8, 5), 5),   # 0 < 2 < 5 -> hold (no scale-down while work)
    ((0, 2, 8, 5), 5),   # min clamp to 2 then hold: never down to MIN_PODS>0
    ((9, 2, 8, 5), 8),   # max clamp
])
def test_clip_truth_table(args, expected):
    assert policy.clip_pod_count(*args) == expected


def test_floor_division_strands_residual_keys():
    # 1 key, KEYS_PER_POD=2 never scales up from 0 (autoscaler.py:217)
    assert policy.desired_for_queue(1, 2, 0, 8, 0) == 0


@pytest.mark.parametrize('keys,min_pods,max_pods,kpp,cur,expected', [
    ({'predict': 1, 'track': 1}, 0, 8, 1, 3, 6),   # multi-queue inflation
    ({'predict': 0, 'track': 0}, 1, 8, 1, 5, 8),   # scale UP on empty queues
    ({'predict': 0, 'track': 0}, 1, 8, 1, 0, 2),   # MIN_PODS per queue
    ({'predict': 3, 'track': 2}, 0, 8, 1, 0, 5),
    ({'predict': 3, 'track': 2}, 0, 8, 2, 0, 2),   # floor per queue
    ({'predict': 20}, 0, 8, 1, 0, 8),              # clamp
    ({'predict': 2}, 0, 8, 1, 6, 6),               # hold
    ({'predict': 0}, 0, 8, 1, 6, 0),               # all-or-nothing down
])
def test_reference_scale_table(keys, min_pods, max_pods, kpp, cur, expected):
    assert policy.decide(keys, min_pods, max_pods, kpp, cur) == expected


def _reference_oracle(keys, min_pods, max_pods, kpp, current):
    """Literal transcription of Autoscaler.scale's arithmetic."""
    def clip(d):
        if d > max_pods:
            d = max_pods
        elif d < min_pods:
            d = min_pods
        if 0 < d < current:
            d = current
        return d
    total = 0
    for q in keys:
        total += clip(keys[q] // kpp)
    return clip(total)


def test_reference_matches_oracle_exhaustively():
    for k1, k2, mn, mx, kpp, cur in itertools.product(
            range(0, 7), range(0, 4), range(0, 3), range(1, 5),
            range(1, 4), range(0, 6)):
        keys = {'predict': k1, 'track': k2}
        assert policy.decide(keys, mn, mx, kpp, cur) == \
            _reference_oracle(keys, mn, mx, kpp, cur)


@pytest.mark.parametrize('keys,min_pods,max_pods,kpp,cur,busy,expected', [
    ({'predict': 1, 'track': 1}, 0, 8, 1, 3, 0, 2),  # global sum, no inflation
    ({'predict': 1}, 0, 8, 2, 0, 0, 1),              # ceil: 1 key -> 1 pod
    ({'predict': 0}, 2, 8, 1, 5, 0, 2),              # may shrink to MIN_PODS
    ({'predict': 0, 'track': 0}, 1, 8, 1, 5, 0, 1),  # no empty-queue scale-up
    ({'predict': 2}, 0, 8, 4, 6, 3, 3),              # never below busy
    ({'predict': 40}, 0, 8, 1, 0, 0, 8),
])
def test_strict_policy(keys, min_pods, max_pods, kpp, cur, busy, expected):
    assert policy.decide(keys, min_pods, max_pods, kpp, cur, policy='strict',
                         busy=busy) == expected


def test_unknown_policy_and_bad_kpp():
    with pytest.raises(ValueError):
        policy.decide({'q': 1}, 0, 1, 1, 0, policy='nope')
    with pytest.raises(ValueError):
        policy.decide({'q': 1}, 0, 1, 0, 0)
