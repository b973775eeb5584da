"""Synthetic key producer: Poisson arrivals during an on-window.

Keys follow the kiosk convention: a job hash (``<queue>:<id>``) is written
first, then its name is ``LPUSH``ed onto the queue -- in one MULTI/EXEC so a
consumer never pops a key whose hash does not exist yet.  The hash carries
``service_ms`` (per-key GPU service time S of BASELINE.md §3), ``rows`` and
the enqueue timestamp (CLOCK_MONOTONIC ns).
"""
import random
import time


def sleep_until_ns(target_ns):
    while True:
        remaining = (target_ns - time.monotonic_ns()) / 1e9
        if remaining <= 0:
            return
        time.sleep(min(remaining, 0.05) if remaining > 0.002 else 0)


class LoadGenerator(object):
    def __init__(self, redis, queues=('predict',), rate=2.0, service_ms=1000,
                 rows=2048, seed=0, prefix='bench'):
        self.redis = redis
        self.queues = list(queues)
        self.rate = float(rate)
        self.service_ms = int(service_ms)
        self.rows = int(rows)
        self.rng = random.Random(seed)
        self.prefix = prefix
        self.counter = 0

    def enqueue(self, queue=None, t_ns=None):
        queue = queue or self.rng.choice(self.queues)
        self.counter += 1
        item = '%s:%s:%d' % (queue, self.prefix, self.counter)
        now = time.monotonic_ns() if t_ns is None else t_ns
        pipe = self.redis.pipeline(transaction=True)
        pipe.hset(item, mapping={'status': 'new', 'service_ms': self.service_ms,
                                 'rows': self.rows, 'seed': self.counter,
                                 'enq_ns': now})
        pipe.lpush(queue, item)
        pipe.execute()
        return item, queue, now

    def on_window(self, t_first_ns, on_s, min_keys=1):
        """Enqueue the first key at ``t_first_ns`` exactly (with
        ``min_keys - 1`` more at once), then Poisson arrivals until the
        window closes.  Returns ``[(item, queue, t)]``."""
        sleep_until_ns(t_first_ns)
        keys = [self.enqueue(t_ns=time.monotonic_ns())
                for _ in range(max(1, int(min_keys)))]
        end = t_first_ns + int(on_s * 1e9)
        t_next = t_first_ns + int(self.rng.expovariate(self.rate) * 1e9)
        while t_next < end:
            sleep_until_ns(t_next)
            keys.append(self.enqueue(t_ns=time.monotonic_ns()))
            t_next += int(self.rng.expovariate(self.rate) * 1e9)
        return keys
