"""amdsmi utilisation sampler: the hardware cross-check of GPU-idle %.

SURVEY §7.4 item 8 / §5.5: the benchmark's GPU-idle % is defined from
worker events (Σ(alive − busy) / Σ alive, busy = a key in flight).  This
samples the firmware's ``gfx_activity`` (percent of time the graphics
engine was busy) through amdsmi while the timed steps run, so the event
-derived busy fraction can be checked against what the GPU itself reports.

amdsmi talks to the kernel driver, never to HIP, so sampling from the
benchmark's rank-0 process does not create a GPU context.  Where amdsmi or
the driver is unavailable (CPU containers) :meth:`UtilSampler.start`
returns ``False`` and the result is ``None``.

It also records what the node holds in HBM: every ``proc_period_s`` each
device's ``vram_used`` (MiB), stamped with ``time.monotonic_ns`` -- the
clock of the lifecycle events -- so :func:`..metrics.hbm_hold` can read the
standby hold at the instants no worker is alive.  (amdsmi's per-process
list reports host-namespace pids, which a container cannot match to its
own processes, so the attribution is by phase, not by pid.)
"""
import threading
import time


class UtilSampler(object):
    def __init__(self, period_s=0.1, bdfs=None, proc_period_s=0.5):
        self.period_s = float(period_s)
        self.proc_period_s = float(proc_period_s)
        self.bdfs = set(b.lower() for b in bdfs) if bdfs else None
        self._thread = None
        self._stop = threading.Event()
        self._samples = {}      # bdf -> [gfx %]
        self.device_vram = {}   # bdf -> [(t_ns, used MiB)]
        self.vram_total_mib = {}
        self._amdsmi = None
        self._handles = []
        self.error = None

    def start(self):
        try:
            import amdsmi
            amdsmi.amdsmi_init()
            handles = []
            for handle in amdsmi.amdsmi_get_processor_handles():
                try:
                    bdf = str(amdsmi.amdsmi_get_gpu_device_bdf(handle)).lower()
                except Exception:  # pylint: disable=broad-except
                    bdf = 'gpu%d' % len(handles)
                if self.bdfs is None or bdf in self.bdfs:
                    handles.append((bdf, handle))
        except Exception as err:  # pylint: disable=broad-except
            self.error = '%s: %s' % (type(err).__name__, err)
            return False
        if not handles:
            self.error = 'no matching GPU handles'
            return False
        self._amdsmi = amdsmi
        self._handles = handles
        self._samples = {bdf: [] for bdf, _ in handles}
        self.device_vram = {bdf: [] for bdf, _ in handles}
        self._thread = threading.Thread(target=self._run, name='amdsmi',
                                        daemon=True)
        self._thread.start()
        return True

    def _run(self):
        next_proc = 0.0
        while not self._stop.is_set():
            for bdf, handle in self._handles:
                try:
                    act = self._amdsmi.amdsmi_get_gpu_activity(handle)
                    value = act.get('gfx_activity')
                    if isinstance(value, (int, float)):
                        self._samples[bdf].append(float(value))
                except Exception:  # pylint: disable=broad-except
                    pass
            if self.proc_period_s > 0 and time.monotonic() >= next_proc:
                next_proc = time.monotonic() + self.proc_period_s
                self._sample_vram()
            self._stop.wait(self.period_s)

    def _sample_vram(self):
        for bdf, handle in self._handles:
            t = time.monotonic_ns()
            try:
                usage = self._amdsmi.amdsmi_get_gpu_vram_usage(handle)
                self.device_vram[bdf].append((t, float(usage['vram_used'])))
                self.vram_total_mib[bdf] = float(usage['vram_total'])
            except Exception:  # pylint: disable=broad-except
                pass

    def vram(self):
        """HBM samples for :func:`..metrics.hbm_hold`."""
        return {'device': {b: list(v) for b, v in self.device_vram.items()},
                'total_mib': dict(self.vram_total_mib)}

    def stop(self):
        """Per-device mean ``gfx_activity`` % (``None`` if never started)."""
        if self._thread is None:
            return None
        self._stop.set()
        self._thread.join(5)
        try:
            self._amdsmi.amdsmi_shut_down()
        except Exception:  # pylint: disable=broad-except
            pass
        out = {}
        for bdf, values in self._samples.items():
            if values:
                out[bdf] = {'gfx_busy_pct': sum(values) / len(values),
                            'samples': len(values)}
        return out


def mean_busy(result):
    """Mean ``gfx_busy_pct`` over devices (``None`` if nothing sampled)."""
    if not result:
        return None
    values = [v['gfx_busy_pct'] for v in result.values()]
    return sum(values) / len(values)


def vram_snapshot(bdfs=None):
    """``{bdf: vram_used MiB}`` right now (``None`` without amdsmi): the
    benchmark's before-anything and after-pool-boot reference points."""
    try:
        import amdsmi
        amdsmi.amdsmi_init()
    except Exception:  # pylint: disable=broad-except
        return None
    wanted = set(b.lower() for b in bdfs) if bdfs else None
    out = {}
    try:
        for handle in amdsmi.amdsmi_get_processor_handles():
            bdf = str(amdsmi.amdsmi_get_gpu_device_bdf(handle)).lower()
            if wanted is None or bdf in wanted:
                out[bdf] = float(
                    amdsmi.amdsmi_get_gpu_vram_usage(handle)['vram_used'])
    except Exception:  # pylint: disable=broad-except
        pass
    finally:
        try:
            amdsmi.amdsmi_shut_down()
        except Exception:  # pylint: disable=broad-except
            pass
    return out or None


def sample_for(seconds, period_s=0.1, bdfs=None, sleep=time.sleep):
    """Convenience: sample for a fixed time (tools, tests)."""
    sampler = UtilSampler(period_s, bdfs)
    if not sampler.start():
        return None
    sleep(seconds)
    return sampler.stop()
