#!/usr/bin/env python3
"""Headline benchmark: scale-up latency (first key -> GPU-ready) and GPU-idle %
of the MI355X autoscaler under bursty Poisson load (BASELINE.json metric).

One *step* = one on/off episode of BASELINE config 4 ("bursty Poisson
arrivals, scale 0 <-> N"): with no worker alive, the first key is enqueued,
Poisson arrivals continue for ``--on`` seconds, the queue drains, the
autoscaler scales back to zero and the standby pool refills.  The whole
product runs for real: ``scale.py`` (the reference-compatible CLI, embedded
GPU manager) spawns PyTorch-ROCm workers pinned to MI355X GPUs, each builds
its random-init model in HBM, runs the gfx950 warm-start kernel, publishes
READY and serves keys with the MFMA MLP (1 s of GPU work per key, S of
BASELINE.md §3), and READY-set changes are fenced with RCCL.

Phase control: the reference's cold-start number is dominated by where the
first key lands in the ``INTERVAL`` tick grid.  Timed episode
``i`` enqueues its first key ``(i + 0.5) / K * INTERVAL`` before the next
tick (stratified sampling of the uniform phase: same expectation as random
phase, far lower variance at small K).  The reference policy with an ideal
(zero-delay) actuator is simulated on the identical arrival trace and
reported beside the measured numbers (``reference_sim``).

Contract: ``python bench.py --gpus N --steps K --warmup W`` (torchrun with
N ranks for N > 1; rank 0 drives, every rank brackets the K timed steps with
barrier + torch.cuda.synchronize(), elapsed = max over ranks).  Scaling is
weak: arrival rate = ``--lam-per-gpu`` x N (0.25/s per GPU -> 2/s at N = 8,
exactly BASELINE config 4) in 60 s bursts (``--on``, config 4's "60 s on");
config 4's 60 s off period is shortened to "until the stack has scaled to
zero, then ``--off`` s", because nothing is measured while no worker is
alive.  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from kiosk_autoscaler_amd.bench import gpu_util  # noqa: E402  (no torch)

METRIC = ('scale-up latency (s) first-key->GPU-ready + GPU-idle-% at fixed '
          'QPS, 1/2/4/8 GPU')
# BASELINE.md §3, QUEUES=predict, MAX_PODS=8, KEYS_PER_POD=1, lam=2/s,
# INTERVAL=5 (BASELINE config 4 at N=8): 3.13 s cold start, 65.6 % idle.
BASELINE_LATENCY_S = 3.13
BASELINE_IDLE_PCT = 65.6
# KIOSK_BENCH_OUT redirects the detail/event files (tests use a tmp dir)
OUT_DIR = os.environ.get('KIOSK_BENCH_OUT') or os.path.join(ROOT, 'gpurun_out')


def log(msg):
    sys.stderr.write('[bench %s] %s\n' % (time.strftime('%H:%M:%S'), msg))
    sys.stderr.flush()


def free_port():
    sock = socket.socket()
    sock.bind(('127.0.0.1', 0))
    port = sock.getsockname()[1]
    sock.close()
    return port


def ensure_built(kernels):
    sys.path.insert(0, os.path.join(ROOT, 'tools'))
    import build_native
    need = not os.path.exists(build_native.KREDIS) or (
        kernels and not os.path.exists(build_native.EXT_PATH))
    if need:
        log('building native components')
        build_native.build(jobs=8, kernels=kernels)
    return build_native.KREDIS


def wait_for(predicate, timeout, step=0.05, what='condition'):
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        value = predicate()
        if value:
            return value
        time.sleep(step)
    raise TimeoutError('timed out waiting for %s' % what)


class Services(object):
    """kredis-server + the autoscaler CLI (embedded GPU manager)."""

    def __init__(self, args, n_gpus):
        self.args = args
        self.n = n_gpus
        self.procs = []
        self.port = free_port()
        os.makedirs(OUT_DIR, exist_ok=True)

    def start(self):
        args = self.args
        kredis = ensure_built(kernels=args.backend == 'hip')
        if os.path.exists(kredis):
            cmd = [kredis, '--port', str(self.port)]
        else:
            cmd = [sys.executable, '-m', 'kiosk_autoscaler_amd.fakes.server',
                   '--port', str(self.port)]
        self.redis_proc = subprocess.Popen(
            cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
            start_new_session=True)
        self.procs.append(self.redis_proc)
        from kiosk_autoscaler_amd.redisq import StrictRedis
        self.redis = StrictRedis(host='127.0.0.1', port=self.port,
                                 decode_responses=True)
        wait_for(lambda: self._ping(), 20, what='redis')
        # the autoscaler and its workers are not torchrun ranks: keep the
        # launcher's rendezvous variables out of their environment
        env = {k: v for k, v in os.environ.items()
               if k not in TORCHRUN_VARS and not k.startswith('TORCHELASTIC')}
        env.update({
            'REDIS_HOST': '127.0.0.1', 'REDIS_PORT': str(self.port),
            'REDIS_INTERVAL': '1', 'QUEUES': args.queues,
            'RESOURCE_NAME': 'bench-worker', 'RESOURCE_NAMESPACE': 'bench',
            'RESOURCE_TYPE': args.resource_type,
            'MIN_PODS': '0', 'MAX_PODS': str(self.n),
            'KEYS_PER_POD': str(args.kpp), 'INTERVAL': str(args.interval),
            'SCALE_POLICY': args.policy,
            'SCALE_DOWN_DELAY': str(args.scale_down_delay),
            'IDLE_INTERVAL': str(args.idle_interval),
            'GPU_IDS': ','.join(str(i) for i in range(self.n)),
            'WORKER_BACKEND': args.backend, 'WARM_POOL': str(self.n),
            'FENCE': args.fence, 'MODEL_DIM': str(args.dim),
            'MODEL_HIDDEN': str(args.hidden), 'MODEL_LAYERS': str(args.layers),
            'ROWS_PER_KEY': str(args.rows), 'EVENT_LOG': 'redis',
            'TICK_KEY': 'kiosk:autoscaler:tick', 'DEBUG': '0',
            'LOG_FILE': os.path.join(OUT_DIR, 'bench_autoscaler.log'),
            'JOB_IDLE_EXIT_S': '0.5',
            'PYTHONPATH': ROOT + os.pathsep + env.get('PYTHONPATH', ''),
        })
        if args.backend == 'cpu':
            env['MOCK_WORK_MS'] = '0'
        self.stdout = open(os.path.join(OUT_DIR, 'bench_autoscaler.out'), 'w')
        self.scaler_proc = subprocess.Popen(
            [sys.executable, os.path.join(ROOT, 'scale.py')], env=env,
            stdout=self.stdout, stderr=subprocess.STDOUT,
            start_new_session=True)
        self.procs.append(self.scaler_proc)
        wait_for(lambda: self.redis.get('kiosk:autoscaler:tick'), 60,
                 what='first autoscaler tick')
        wait_for(self.pool_ready, args.pool_timeout, step=0.2,
                 what='standby pool boot')
        return self

    def _ping(self):
        try:
            return self.redis.ping()
        except Exception:  # pylint: disable=broad-except
            return False

    def pool_ready(self):
        if self.scaler_proc.poll() is not None:
            raise RuntimeError('autoscaler exited with %s (see %s)' % (
                self.scaler_proc.returncode, self.stdout.name))
        value = self.redis.get('kiosk:pool')
        if not value:
            return False
        booted, _total = (int(v) for v in value.split())
        return booted >= self.n

    def idle(self):
        if any(True for _ in self.redis.scan_iter(match='kiosk:worker:*')):
            return False
        for queue in self.args.queues.split(','):
            if self.redis.llen(queue):
                return False
            if any(True for _ in self.redis.scan_iter(
                    match='processing-%s:*' % queue)):
                return False
        return self.pool_ready()

    def next_tick_ns(self):
        start, end, _ = (int(v) for v in
                         self.redis.get('kiosk:autoscaler:tick').split())
        period = int(self.args.interval * 1e9) + (end - start)
        nxt = end + int(self.args.interval * 1e9)
        return nxt, period

    def stop(self):
        if getattr(self, 'scaler_proc', None) is not None and \
                self.scaler_proc.poll() is None:
            self.scaler_proc.send_signal(signal.SIGTERM)
            try:
                self.scaler_proc.wait(timeout=60)
            except subprocess.TimeoutExpired:
                os.killpg(self.scaler_proc.pid, signal.SIGKILL)
        for proc in self.procs:
            if proc.poll() is None:
                try:
                    os.killpg(proc.pid, signal.SIGTERM)
                    proc.wait(timeout=10)
                except (OSError, subprocess.TimeoutExpired):
                    proc.kill()
        if getattr(self, 'stdout', None):
            self.stdout.close()


def run_episode(svc, gen, args, delay_s, tag):
    """One on/off episode whose first key lands ``delay_s`` before a tick."""
    wait_for(svc.idle, args.idle_timeout, step=0.1, what='idle before ' + tag)
    nxt, period = svc.next_tick_ns()
    now = time.monotonic_ns()
    target = nxt - int(delay_s * 1e9)
    while target < now + int(0.05e9):
        nxt += period
        target = nxt - int(delay_s * 1e9)
    keys = gen.on_window(target, args.on)
    t_first = keys[0][2]
    items = [k[0] for k in keys]

    def all_done():
        pipe = svc.redis.pipeline(transaction=False)
        for item in items:
            pipe.hget(item, 'status')
        return all(s == 'done' for s in pipe.execute())
    wait_for(all_done, args.drain_timeout, step=0.1, what='drain ' + tag)
    t_done = time.monotonic_ns()
    wait_for(svc.idle, args.idle_timeout, step=0.1, what='scale-down ' + tag)
    t_idle = time.monotonic_ns()
    off_left = args.off - (t_idle - t_done) / 1e9
    if off_left > 0:
        time.sleep(off_left)
    log('%s: %d keys, delay %.2fs, drained %.1fs after first key, idle '
        '%.1fs' % (tag, len(keys), delay_s, (t_done - t_first) / 1e9,
                   (t_idle - t_first) / 1e9))
    return {'t_first': t_first, 't_end': t_idle, 'keys': keys,
            'delay_s': delay_s, 'tick_ns': nxt}


def reference_sim(episodes, args):
    """The reference policy + ideal actuator on each episode's trace."""
    from kiosk_autoscaler_amd.bench import sim
    results = []
    for ep in episodes:
        offset = args.interval - ep['delay_s']
        arrivals = [((t - ep['t_first']) / 1e9 + offset, q)
                    for _, q, t in ep['keys']]
        results.append(sim.simulate(
            arrivals, interval=args.interval, service_s=args.service_ms / 1e3,
            ready_delay=0.0, max_pods=args.n_gpus, keys_per_pod=args.kpp,
            queues=args.queues.split(','), policy='reference',
            tick_s=0.0, first_tick=0.0))
    lat = [r['cold_start_mean_s'] for r in results if r['cold_start_mean_s']]
    idle = [r['gpu_idle_pct'] for r in results if r['gpu_idle_pct']]
    return {'latency_mean_s': sum(lat) / len(lat) if lat else None,
            'gpu_idle_pct': sum(idle) / len(idle) if idle else None,
            'ready_delay_s': 0.0}


def parse_args():
    p = argparse.ArgumentParser(description=__doc__.split('\n')[0])
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=3)
    p.add_argument('--warmup', type=int, default=1)
    p.add_argument('--interval', type=float, default=5.0)
    p.add_argument('--lam-per-gpu', type=float, default=0.25)
    p.add_argument('--on', type=float, default=60.0)
    p.add_argument('--off', type=float, default=2.0)
    p.add_argument('--service-ms', type=int, default=1000)
    p.add_argument('--queues', default='predict')
    p.add_argument('--kpp', type=int, default=1)
    p.add_argument('--policy', default='reference')
    p.add_argument('--scale-down-delay', type=float, default=0.0)
    p.add_argument('--idle-interval', type=float, default=0.0,
                   help='opt-in fast poll while at zero workers (changes the '
                        "reference's INTERVAL semantics; reported separately)")
    p.add_argument('--resource-type', default='deployment')
    p.add_argument('--backend', default='hip')
    p.add_argument('--fence', default='auto')
    p.add_argument('--dim', type=int, default=4096)
    p.add_argument('--hidden', type=int, default=16384)
    p.add_argument('--layers', type=int, default=4)
    p.add_argument('--rows', type=int, default=2048)
    p.add_argument('--seed', type=int, default=2024)
    p.add_argument('--pool-timeout', type=float, default=240.0)
    p.add_argument('--idle-timeout', type=float, default=120.0)
    p.add_argument('--drain-timeout', type=float, default=300.0)
    return p.parse_args()


TORCHRUN_VARS = ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'LOCAL_WORLD_SIZE',
                 'GROUP_RANK', 'GROUP_WORLD_SIZE', 'ROLE_RANK', 'ROLE_NAME',
                 'ROLE_WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT',
                 'OMP_NUM_THREADS_SET')


def main():
    args = parse_args()
    rank = int(os.environ.get('RANK', 0))
    world = int(os.environ.get('WORLD_SIZE', 1))
    local_rank = int(os.environ.get('LOCAL_RANK', 0))
    args.n_gpus = args.gpus
    svc = None
    if rank == 0:
        # everything that forks runs before this process touches the GPU
        svc = Services(args, args.gpus).start()
        log('services up: redis :%d, standby pool booted' % svc.port)
    import torch
    dist = None
    if world > 1:
        import datetime
        import torch.distributed as dist
        dist.init_process_group('gloo', rank=rank, world_size=world,
                                timeout=datetime.timedelta(hours=3))
    use_cuda = torch.cuda.is_available() and args.backend == 'hip'
    if use_cuda:
        torch.cuda.set_device(local_rank)

    def barrier():
        if dist is not None:
            dist.barrier()

    def sync():
        if use_cuda:
            torch.cuda.synchronize()

    episodes = []
    try:
        barrier()
        if rank == 0:
            from kiosk_autoscaler_amd.bench.loadgen import LoadGenerator
            gen = LoadGenerator(svc.redis, args.queues.split(','),
                                rate=args.lam_per_gpu * args.gpus,
                                service_ms=args.service_ms, rows=args.rows,
                                seed=args.seed)
            for w in range(args.warmup):
                run_episode(svc, gen, args, 0.5 * args.interval,
                            'warmup %d' % w)
        sampler = None
        if rank == 0:
            sampler = start_util_sampler(args.gpus)
        barrier()
        sync()
        t0 = time.perf_counter()
        if rank == 0:
            for i in range(args.steps):
                delay = (i + 0.5) / args.steps * args.interval
                episodes.append(run_episode(svc, gen, args, delay,
                                            'step %d' % i))
        sync()
        barrier()
        elapsed = time.perf_counter() - t0
        util = sampler.stop() if sampler is not None else None
        if dist is not None:
            tensor = torch.tensor([elapsed], dtype=torch.float64)
            dist.all_reduce(tensor, op=dist.ReduceOp.MAX)
            elapsed = float(tensor.item())
        if rank == 0:
            from kiosk_autoscaler_amd.bench import metrics
            from kiosk_autoscaler_amd.utils.events import drain_redis
            events = drain_redis(svc.redis)
            summary = metrics.summarize(events, episodes)
            ref = reference_sim(episodes, args)
            from kiosk_autoscaler_amd.bench import sim
            derived = sim.derived_baseline(
                args.lam_per_gpu * args.gpus, args.gpus, args.kpp,
                args.queues.split(','), args.interval, args.service_ms / 1e3)
            value = summary['latency_mean_s']
            detail = {'summary': summary, 'reference_sim': ref,
                      'derived_baseline': derived,
                      'args': vars(args), 'amdsmi': util,
                      'amdsmi_error': getattr(sampler, 'error', None)}
            with open(os.path.join(OUT_DIR, 'bench_detail_n%d.json' %
                                   args.gpus), 'w') as handle:
                json.dump(detail, handle, indent=1, default=str)
            with open(os.path.join(OUT_DIR, 'bench_events_n%d.jsonl' %
                                   args.gpus), 'w') as handle:
                for event in events:
                    handle.write(json.dumps(event) + '\n')
            line = {
                'metric': METRIC,
                'value': round(value, 4) if value is not None else None,
                'unit': 's',
                'n_gpus': args.gpus,
                'steps': args.steps,
                'warmup': args.warmup,
                'ms_per_step': round(elapsed * 1e3 / max(1, args.steps), 1),
                'higher_is_better': False,
                'scaling': 'weak',
                'vs_baseline': (round(value / BASELINE_LATENCY_S, 4)
                                if value is not None else None),
                'dtype': 'bf16',
                'data': 'synthetic Poisson on/off keys; random-init weights',
                'config': {
                    'model': 'kiosk-mlp %dx(%d->%d->%d) bf16' % (
                        args.layers, args.dim, args.hidden, args.dim),
                    'global_batch': args.rows, 'seq_len': 1,
                    'parallelism': 'replica-dp%d' % args.gpus,
                    'queues': args.queues, 'interval_s': args.interval,
                    'lambda_per_s': args.lam_per_gpu * args.gpus,
                    'on_s': args.on,
                    'off': 'until scaled to zero, then %g s' % args.off,
                    'service_s': args.service_ms / 1e3,
                    'max_pods': args.gpus, 'keys_per_pod': args.kpp,
                    'policy': args.policy, 'resource_type': args.resource_type,
                    'idle_interval_s': args.idle_interval,
                },
                'gpu_idle_pct': _r(summary['gpu_idle_pct']),
                'baseline_gpu_idle_pct': BASELINE_IDLE_PCT,
                'cold_starts': summary['cold_starts'],
                'first_key_latency_mean_s': _r(
                    summary['first_key_latency_mean_s']),
                'latency_p50_s': _r(summary['latency_p50_s']),
                'latency_max_s': _r(summary['latency_max_s']),
                'decision_mean_s': _r(summary['decision_mean_s']),
                'actuation_mean_s': _r(summary['actuation_mean_s']),
                'first_result_mean_s': _r(summary['first_result_mean_s']),
                'queue_wait_mean_s': _r(summary['queue_wait_mean_s']),
                'keys_done': summary['keys_done'], 'keys': summary['keys'],
                # hardware cross-check of the event-derived busy fraction
                'event_busy_wall_pct': _r(100.0 * summary['gpu_busy_s'] /
                                          max(1e-9, elapsed * args.gpus)),
                'amdsmi_gfx_busy_pct': _r(gpu_util.mean_busy(util)),
                'fence': {k: _r(v) for k, v in summary['fence'].items()},
                'reference_sim_latency_s': _r(ref['latency_mean_s']),
                # same arrival trace, reference policy, ideal zero-delay
                # actuator: the like-for-like comparison (BASELINE.md's
                # 3.13 s comes from a different trace)
                'vs_reference_sim_same_trace': (
                    round(value / ref['latency_mean_s'], 4)
                    if value is not None and ref['latency_mean_s'] else None),
                'reference_sim_gpu_idle_pct': _r(ref['gpu_idle_pct']),
                # BASELINE.md's method (1200 s, 60/60 on/off, 5 seeds) at
                # this N's lambda and MAX_PODS: the per-N reference curve
                'derived_baseline_latency_s': _r(derived['latency_mean_s']),
                'derived_baseline_gpu_idle_pct': _r(derived['gpu_idle_pct']),
            }
            print(json.dumps(line), flush=True)
    finally:
        if svc is not None:
            svc.stop()
        if dist is not None:
            dist.destroy_process_group()


def start_util_sampler(n_gpus):
    """amdsmi gfx-activity sampling over the managed GPUs (None on CPU)."""
    if os.environ.get('KIOSK_AMDSMI', '1') == '0':
        return None
    bdfs = None
    try:
        from kiosk_autoscaler_amd.gpumgr import gpus
        slots = gpus.discover(','.join(str(i) for i in range(n_gpus)),
                              env={}, cpu_slots=0)
        found = [s.pci for s in slots if getattr(s, 'pci', None)]
        if len(found) == n_gpus:
            bdfs = found
    except Exception:  # pylint: disable=broad-except
        pass
    sampler = gpu_util.UtilSampler(0.1, bdfs)
    sampler.start()
    return sampler


def _r(value, nd=4):
    return round(value, nd) if isinstance(value, float) else value


if __name__ == '__main__':
    main()
