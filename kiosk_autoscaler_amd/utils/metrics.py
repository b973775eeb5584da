"""Optional Prometheus exporter (``METRICS_PORT``).

The reference has no metrics endpoint (its only telemetry is the INFO log
lines of ``autoscaler/autoscaler.py:77,239-241``).  Here the autoscaler and
the manager daemon can serve ``/metrics``:

* from the event stream (an :class:`~.events.EventLog` observer): queue
  depth and in-flight keys per queue, desired / current workers, tick
  duration, scale events, assignment -> READY latency, worker exits by
  outcome, requeued items, watchdog kills, fence epochs and their duration,
  node-communicator generations / shrinks / breaks / fallbacks / hung-rank
  kills and their init times, process spawns (zygote fork or exec),
  free-HBM sizing;
* at scrape time from the GPU manager: workers per state, standbys
  (booted / booting), GPU slots, READY vs fenced (available) replicas per
  resource, the node communicator's state and rank count.

``prometheus_client`` is imported only when the exporter is enabled.
"""
import logging

logger = logging.getLogger('Metrics')

LATENCY_BUCKETS = (0.002, 0.005, 0.01, 0.02, 0.05, 0.1, 0.25, 0.5, 1.0,
                   2.5, 5.0, 10.0, 30.0)


class PrometheusExporter(object):
    def __init__(self, port=0, addr='0.0.0.0', manager=None, serve=True):
        from prometheus_client import (CollectorRegistry, Counter, Gauge,
                                       Histogram, start_http_server)
        self.registry = CollectorRegistry()
        r = self.registry
        self.queue_keys = Gauge('kiosk_queue_keys', 'LLEN + in-flight keys '
                                'per queue (the tally)', ['queue'],
                                registry=r)
        self.in_progress = Gauge('kiosk_in_progress_keys', 'processing-* '
                                 'keys per queue', ['queue'], registry=r)
        self.desired = Gauge('kiosk_desired_workers', 'decision of the '
                             'last tick', registry=r)
        self.current = Gauge('kiosk_current_workers', 'declared workers '
                             'seen by the last tick', registry=r)
        self.ticks = Counter('kiosk_ticks', 'reconcile ticks', registry=r)
        self.tick_seconds = Histogram('kiosk_tick_seconds', 'tally + '
                                      'decision time', registry=r,
                                      buckets=LATENCY_BUCKETS)
        self.scales = Counter('kiosk_scale_events', 'actuations',
                              ['direction'], registry=r)
        self.ready_seconds = Histogram(
            'kiosk_worker_ready_seconds', 'assignment -> READY',
            ['from_pool'], registry=r, buckets=LATENCY_BUCKETS)
        self.exits = Counter('kiosk_worker_exits', 'worker exits by outcome',
                             ['outcome'], registry=r)
        self.requeued = Counter('kiosk_requeued_items', 'in-flight items '
                                'pushed back after a worker death',
                                registry=r)
        self.timeouts = Counter('kiosk_watchdog_kills', 'hung workers '
                                'killed by the watchdog', registry=r)
        self.fences = Counter('kiosk_fence_epochs', 'membership fences',
                              ['transport'], registry=r)
        self.fence_seconds = Histogram('kiosk_fence_seconds', 'fence epoch '
                                       'start -> rank-0 ack', registry=r,
                                       buckets=LATENCY_BUCKETS)
        self.comm_builds = Counter('kiosk_node_comm_generations',
                                   'node communicators built (pool boot, '
                                   'regrows, rebuilds after a break)',
                                   registry=r)
        self.comm_shrinks = Counter('kiosk_node_comm_shrinks', 'lost ranks '
                                    'shrunk out of the node communicator',
                                    registry=r)
        self.comm_shrink_seconds = Histogram(
            'kiosk_node_comm_shrink_seconds', 'slowest survivor of a shrink',
            registry=r, buckets=LATENCY_BUCKETS)
        self.comm_fallbacks = Counter('kiosk_node_comm_fallbacks', 'switches '
                                      'to the fallback transport',
                                      ['transport'], registry=r)
        self.hung_kills = Counter('kiosk_node_rank_hung_kills', 'ranks '
                                  'killed for not answering a failed '
                                  'connect / fence', registry=r)
        self.spawns = Counter('kiosk_process_spawns', 'worker / standby '
                              'processes started', ['via'], registry=r)
        self.comm_breaks = Counter('kiosk_node_comm_breaks', 'node '
                                   'communicator generations dropped',
                                   ['failed'], registry=r)
        self.comm_init_seconds = Histogram(
            'kiosk_node_comm_init_seconds', 'slowest rank of a generation',
            registry=r, buckets=LATENCY_BUCKETS)
        self.hbm_free = Gauge('kiosk_hbm_free_bytes', 'free HBM a standby '
                              'measured at its last assignment', ['gpu'],
                              registry=r)
        self.kpp = Gauge('kiosk_keys_per_pod_effective', 'KEYS_PER_POD '
                         'after free-HBM sizing', ['gpu'], registry=r)
        self.pool_parks = Counter('kiosk_pool_parks', 'deep idle: standby '
                                  'pool released', registry=r)
        self.pool_wakes = Counter('kiosk_pool_wakes', 'parked pool refilled',
                                  ['reason'], registry=r)
        self.prebuild_seconds = Histogram(
            'kiosk_standby_prebuild_seconds', 'arrival-woken standby: engine '
            'prebuilt before the assignment', registry=r,
            buckets=LATENCY_BUCKETS)
        if manager is not None:
            r.register(_ManagerCollector(manager))
        self.port = None
        if serve:
            server = start_http_server(port, addr=addr, registry=r)
            # prometheus_client >= 0.17 returns (server, thread)
            if isinstance(server, tuple):
                server = server[0]
            self.port = server.server_address[1] if server else port
            logger.info('Prometheus metrics on %s:%s/metrics', addr,
                        self.port)

    def observe(self, record):
        ev = record.get('ev')
        if ev == 'tick':
            self.ticks.inc()
            for queue, n in (record.get('keys') or {}).items():
                self.queue_keys.labels(queue).set(n)
            for queue, n in (record.get('in_progress') or {}).items():
                self.in_progress.labels(queue).set(n)
            self.desired.set(record.get('desired') or 0)
            self.current.set(record.get('current') or 0)
            if record.get('tick_s') is not None:
                self.tick_seconds.observe(record['tick_s'])
        elif ev == 'scale':
            up = (record.get('desired') or 0) > (record.get('current') or 0)
            self.scales.labels('up' if up else 'down').inc()
        elif ev == 'worker_up':
            self.ready_seconds.labels(
                str(bool(record.get('from_pool'))).lower()).observe(
                    record.get('ready_s') or 0.0)
        elif ev == 'worker_exit':
            if record.get('recycled'):
                outcome = 'recycled'
            elif record.get('killed'):
                outcome = 'killed'
            elif record.get('code') == 0:
                outcome = 'clean'
            else:
                outcome = 'failed'
            self.exits.labels(outcome).inc()
        elif ev == 'requeue':
            self.requeued.inc(record.get('items') or 0)
        elif ev == 'worker_timeout':
            self.timeouts.inc()
        elif ev == 'fence_done':
            self.fences.labels(str(record.get('transport'))).inc()
            if record.get('wall_s') is not None:
                self.fence_seconds.observe(record['wall_s'])
        elif ev == 'node_comm_ready':
            seconds = float(record.get('init_ms') or 0.0) / 1e3
            if record.get('mode') == 'shrink':
                self.comm_shrinks.inc()
                self.comm_shrink_seconds.observe(seconds)
            else:
                self.comm_builds.inc()
                self.comm_init_seconds.observe(seconds)
        elif ev == 'node_comm_fallback':
            self.comm_fallbacks.labels(str(record.get('transport'))).inc()
        elif ev == 'node_rank_hung':
            self.hung_kills.inc()
        elif ev == 'process_spawn':
            self.spawns.labels(str(record.get('via') or 'exec')).inc()
        elif ev == 'node_comm_break':
            self.comm_breaks.labels(
                str(bool(record.get('failed'))).lower()).inc()
        elif ev == 'pool_parked':
            self.pool_parks.inc()
        elif ev == 'pool_resumed':
            self.pool_wakes.labels(str(record.get('reason') or 'demand')).inc()
        elif ev == 'standby_prebuilt' and not record.get('error'):
            self.prebuild_seconds.observe(float(record.get('ms') or 0.0) / 1e3)
        elif ev == 'hbm_sizing':
            gpu = str(record.get('gpu'))
            self.hbm_free.labels(gpu).set(record.get('hbm_free') or 0)
            self.kpp.labels(gpu).set(record.get('keys_per_pod') or 0)


class _ManagerCollector(object):
    """Scrape-time view of the GPU manager's state."""

    def __init__(self, manager):
        self.manager = manager

    def collect(self):
        from prometheus_client.core import GaugeMetricFamily
        try:
            status = self.manager.status()
        except Exception:  # pylint: disable=broad-except
            return
        workers = GaugeMetricFamily('kiosk_workers', 'live workers by state',
                                    labels=['resource', 'state'])
        for res in status.get('resources', []):
            counts = {}
            for w in res.get('workers', []):
                counts[w['state']] = counts.get(w['state'], 0) + 1
            for state in ('starting', 'ready', 'draining'):
                workers.add_metric([res['metadata']['name'], state],
                                   counts.get(state, 0))
        yield workers
        standbys = GaugeMetricFamily('kiosk_standbys', 'warm-pool processes',
                                     labels=['booted'])
        sb = status.get('standbys', [])
        standbys.add_metric(['true'], sum(1 for p in sb if p['booted']))
        standbys.add_metric(['false'], sum(1 for p in sb if not p['booted']))
        yield standbys
        yield GaugeMetricFamily('kiosk_gpu_slots', 'GPU slots managed',
                                value=len(status.get('slots', [])))
        pool = status.get('pool') or {}
        yield GaugeMetricFamily('kiosk_pool_parked', 'deep idle: the standby '
                                'pool is released (1) or resident (0)',
                                value=1 if pool.get('parked') else 0)
        if pool.get('queue_reads') is not None:
            from prometheus_client.core import CounterMetricFamily
            reads = CounterMetricFamily(
                'kiosk_manager_queue_reads', 'LLEN commands the manager '
                'issued to watch the queues (arrival wake, demand sizing), '
                'inside / outside the wake window', labels=['window'])
            fine = pool.get('queue_reads_fine') or 0
            reads.add_metric(['inside'], fine)
            reads.add_metric(['outside'], pool['queue_reads'] - fine)
            yield reads
        if pool.get('wake_lead_s') is not None:
            yield GaugeMetricFamily('kiosk_pool_wake_lead_seconds', 'how '
                                    'long before the next tick an arrival '
                                    'wakes the parked pool',
                                    value=pool['wake_lead_s'])
        replicas = GaugeMetricFamily(
            'kiosk_replicas', 'per resource: READY workers vs the READY '
            'workers of the last fenced membership (available)',
            labels=['resource', 'kind'])
        for res in status.get('resources', []):
            st = res.get('status') or {}
            name = res['metadata']['name']
            replicas.add_metric([name, 'ready'],
                                st.get('ready_replicas') or 0)
            replicas.add_metric([name, 'available'],
                                st.get('available_replicas') or 0)
        yield replicas
        node = status.get('node_comm')
        if node:
            yield GaugeMetricFamily('kiosk_node_comm_ranks', 'ranks of the '
                                    'current node communicator',
                                    value=node.get('ranks') or 0)
            state = GaugeMetricFamily('kiosk_node_comm_state', 'node '
                                      'communicator state (1 = current)',
                                      labels=['state'])
            for name in ('none', 'init', 'ready', 'shrink'):
                state.add_metric([name], 1 if node.get('state') == name
                                 else 0)
            yield state


def attach(events, port, manager=None, addr='0.0.0.0'):
    """Start the exporter and subscribe it to ``events``; returns it (or
    ``None`` when ``port`` is 0 or prometheus_client is missing)."""
    if not port:
        return None
    try:
        exporter = PrometheusExporter(port, addr=addr, manager=manager)
    except ImportError as err:
        logger.error('METRICS_PORT set but prometheus_client is missing: %s',
                     err)
        return None
    events.observers.append(exporter.observe)
    return exporter
