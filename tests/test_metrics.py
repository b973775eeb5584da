"""Prometheus exporter (METRICS_PORT): event-fed counters/histograms and the
scrape-time manager collector."""
import urllib.request

import pytest

pytest.importorskip('prometheus_client')

from kiosk_autoscaler_amd import gpumgr  # noqa: E402
from kiosk_autoscaler_amd.gpumgr import gpus  # noqa: E402
from kiosk_autoscaler_amd.utils import metrics  # noqa: E402
from kiosk_autoscaler_amd.utils.events import EventLog  # noqa: E402


def test_exporter_counts_events_and_serves_http():
    from prometheus_client import generate_latest
    slots = [gpus.GpuSlot(i, '', kind='cpu') for i in range(3)]
    manager = gpumgr.GpuManager(slots, fence=False)
    manager.register('deployment', 'ns', 'w',
                     gpumgr.WorkerTemplate(queues=['q'], backend='cpu'))
    events = EventLog(source='test')
    # port 0 = an ephemeral port here (METRICS_PORT=0 itself means "off")
    exporter = metrics.PrometheusExporter(0, addr='127.0.0.1',
                                          manager=manager)
    events.observers.append(exporter.observe)
    events.emit('tick', keys={'q': 4}, in_progress={'q': 1}, current=1,
                desired=3, tick_s=0.002)
    events.emit('scale', current=1, desired=3)
    events.emit('worker_up', ready_s=0.009, from_pool=True)
    events.emit('worker_exit', code=0, recycled=True)
    events.emit('worker_exit', code=-9, killed='no progress')
    events.emit('requeue', items=2)
    events.emit('fence_done', transport='rccl', wall_s=0.05)
    events.emit('node_comm_ready', gen=1, n=8, init_ms=1900.0, mode='init')
    events.emit('node_comm_ready', gen=1, sub=1, n=7, init_ms=3.0,
                mode='shrink')
    events.emit('node_comm_break', gen=1, failed=False)
    events.emit('node_comm_fallback', gen=2, transport='shm')
    events.emit('node_rank_hung', gen=2, slot=3, pid=1)
    events.emit('process_spawn', pid=1, via='zygote')
    events.emit('process_spawn', pid=2)
    events.emit('hbm_sizing', gpu=0, hbm_free=2.8e11, keys_per_pod=4)
    events.emit('pool_parked', standbys=1, idle_s=0.5)
    events.emit('pool_resumed', reason='arrival')
    events.emit('pool_resumed')
    events.emit('standby_prebuilt', ms=11.0, error=None)
    text = generate_latest(exporter.registry).decode()
    for line in ('kiosk_node_comm_generations_total 1.0',
                 'kiosk_node_comm_breaks_total{failed="false"} 1.0',
                 'kiosk_node_comm_init_seconds_count 1.0',
                 'kiosk_node_comm_shrinks_total 1.0',
                 'kiosk_node_comm_shrink_seconds_count 1.0',
                 'kiosk_node_comm_fallbacks_total{transport="shm"} 1.0',
                 'kiosk_node_rank_hung_kills_total 1.0',
                 'kiosk_process_spawns_total{via="zygote"} 1.0',
                 'kiosk_process_spawns_total{via="exec"} 1.0',
                 'kiosk_hbm_free_bytes{gpu="0"} 2.8e+11',
                 'kiosk_keys_per_pod_effective{gpu="0"} 4.0',
                 'kiosk_pool_parks_total 1.0',
                 'kiosk_pool_wakes_total{reason="arrival"} 1.0',
                 'kiosk_pool_wakes_total{reason="demand"} 1.0',
                 'kiosk_standby_prebuild_seconds_count 1.0'):
        assert line in text, line
    for line in ('kiosk_queue_keys{queue="q"} 4.0',
                 'kiosk_in_progress_keys{queue="q"} 1.0',
                 'kiosk_desired_workers 3.0',
                 'kiosk_scale_events_total{direction="up"} 1.0',
                 'kiosk_worker_ready_seconds_count{from_pool="true"} 1.0',
                 'kiosk_worker_exits_total{outcome="recycled"} 1.0',
                 'kiosk_worker_exits_total{outcome="killed"} 1.0',
                 'kiosk_requeued_items_total 2.0',
                 'kiosk_fence_epochs_total{transport="rccl"} 1.0',
                 'kiosk_gpu_slots 3.0',
                 'kiosk_pool_parked 0.0',
                 'kiosk_workers{resource="w",state="ready"} 0.0',
                 'kiosk_replicas{kind="ready",resource="w"} 0.0',
                 'kiosk_replicas{kind="available",resource="w"} 0.0'):
        assert line in text, line
    if exporter.port:
        body = urllib.request.urlopen(
            'http://127.0.0.1:%d/metrics' % exporter.port, timeout=5).read()
        assert b'kiosk_ticks_total 1.0' in body


def test_disabled_is_free():
    events = EventLog(source='test')
    assert metrics.attach(events, port=0) is None
    assert events.observers == []
