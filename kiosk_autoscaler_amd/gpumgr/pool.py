"""The standby pool of the node-local GPU manager:
warm standby processes pinned to the GPUs the next scale-up takes, the
worker zygote they fork from, deep idle (park / arrival wake / wake lead),
recycling of drained workers, PCI verification of each slot, and reaping.

A mixin of :class:`~.controller.GpuManager` (shared lock, events, slots and
resources); split out of ``controller.py``.  Every
method runs under the manager lock.
"""
import collections
import json
import logging
import os
import subprocess
import time

from .. import policy
from .nodecomm import NODE_EVENTS
from .process import (DRAINING, EXITED, ManagedProcess, Pipe,
                      bare_worker)

logger = logging.getLogger('GpuManager')

POOL_KEY = 'kiosk:pool'
SLOTS_KEY = 'kiosk:slots'


class PoolMixin(object):
    """Standbys, zygote, deep idle, recycling (see the module doc)."""

    def _init_pool(self, pool_size, pool_template, pool_mode, recycle,
                   pool_idle_release_s, pool_wake_poll_s, pool_wake_hold_s,
                   pool_wake_lead_s, zygote):
        self.pool_size = max(0, int(pool_size))
        self.pool_template = pool_template
        self.pool_mode = pool_mode
        self.recycle = bool(recycle)
        self.retiring = []   # recycled processes told to exit
        self.standbys = collections.OrderedDict()   # slot index -> process
        # deep idle: after this long without demand the standbys exit and
        # the pool stays empty until the next scale-up (0 = never)
        self.pool_idle_release_s = float(pool_idle_release_s or 0.0)
        self.pool_parked = False
        self.pool_parks = 0
        self._last_demand = time.monotonic()
        self.pool_wake_poll_s = float(pool_wake_poll_s or 0.0)
        self.pool_wake_hold_s = float(pool_wake_hold_s or 0.0)
        self._wake_until = 0.0
        self.pool_wake_lead_s = float(pool_wake_lead_s or 0.0)
        self._next_tick = None    # monotonic instant of the next tick
        # spawn request -> booted+prebuilt of recent arrival-woken standbys:
        # the lead adapts to it (wake_lead)
        self._wake_boots = collections.deque(maxlen=16)
        self._wake_at = None      # a deferred arrival wake
        self.wake_deferrals = 0   # wakes skipped: the tick would not scale
        if not hasattr(self, 'wake_policy'):
            self.wake_policy = None
        self._spawn_at = None     # a deferred standby spawn (awake pool)
        self._park_at = None      # when an idle pool is due to park
        self._next_arrival_check = 0.0
        self._arrival_watch = False   # no demand: queues are polled
        # queue -> length at the last check; reset to empty when demand
        # ends (a scale to zero implies empty queues, stranded keys aside),
        # so a key landing before the first check still counts as arrived
        self._queued = {}
        # keys waiting in the managed queues at the last reading: a
        # deep-idle pool keeps a standby per KEYS_PER_POD of them
        self._waiting = 0
        self._waiting_by_queue = {}
        self._next_waiting_check = 0.0
        self.arrival_wakes = 0
        # LLEN commands this manager issued for the pool (arrival watch and
        # demand sizing), and how many of them fell inside a wake window:
        # the standing Redis load of an idle node
        self.queue_reads = 0
        self.queue_reads_fine = 0
        # worker zygote (worker/zygote.py): spawns fork from a process that
        # imported the worker (and torch, for a plug-in) without the GPU
        self.zygote_enabled = bool(zygote)
        self.zygote = None
        self._zygote_restart_at = 0.0
        self.mapping_fixes = 0   # slots remapped after a PCI check
        self._orphan_scan_at = 0.0
        self._zombies_seen = set()

    # ------------------------------------------------------------------
    # process management
    # ------------------------------------------------------------------
    @staticmethod
    def _interpreter(template):
        argv = [template.python]
        if bare_worker(template):
            # the torch-free HIP worker needs only this tree (on PYTHONPATH
            # below) and the stdlib: skipping site-packages' .pth
            # processing takes ~20 ms off every spawn
            argv.append('-S')
        return argv

    def _environment(self, template):
        env = dict(os.environ)
        if getattr(self, 'hw_queues', 0):
            # WORKER_HW_QUEUES (a template's own setting still wins)
            env['GPU_MAX_HW_QUEUES'] = str(self.hw_queues)
        env.update({k: str(v) for k, v in template.env.items()})
        # the RCCL library the node ladder is on now: loaded first by a new
        # process's preload (the manager's own environment stays as it was)
        lib = self.node.current_lib() if self.node is not None else None
        if lib:
            env['KIOSK_RCCL_LIB'] = lib
        env['PYTHONUNBUFFERED'] = '1'
        root = os.path.dirname(os.path.dirname(os.path.dirname(
            os.path.abspath(__file__))))
        env['PYTHONPATH'] = os.pathsep.join(
            [root] + [p for p in env.get('PYTHONPATH', '').split(os.pathsep)
                      if p])
        return env
    # env that decides what a worker imports: a zygote serves only the
    # templates it preloaded for
    _IMPORT_ENV = ('WORKER_ENGINE', 'WORKER_IMPORT_TORCH', 'KIOSK_NATIVE')

    def _start_zygote(self):
        tpl = self.pool_template
        if not self.zygote_enabled or tpl is None or self.zygote is not None \
                or tpl.module != 'kiosk_autoscaler_amd.worker.main' or \
                self._stopping or time.monotonic() < self._zygote_restart_at:
            return
        from ..worker import zygote
        if not zygote.become_subreaper():
            logger.warning('PR_SET_CHILD_SUBREAPER refused: no zygote.')
            self.zygote_enabled = False
            return
        argv = self._interpreter(tpl) + [
            '-m', 'kiosk_autoscaler_amd.worker.zygote', '--backend',
            tpl.backend]
        rocr = self._rocr_embryos = self.zygote_rocr_embryos(tpl)
        # each ROCr embryo initialises one GPU only (lowest slots first: the
        # slots a scale-up takes first)
        gpus = self._distinct_gpus()[:rocr]
        self.zygote = zygote.ZygoteClient(argv, self._environment(tpl),
                                          embryos=self.zygote_embryos(),
                                          rocr_embryos=rocr, rocr_gpus=gpus)
        self.events.emit('zygote_spawn', pid=self.zygote.pid,
                         embryos=self.zygote_embryos(), rocr_embryos=rocr,
                         rocr_gpus=gpus)

    def zygote_embryos(self):
        """Pre-forked workers the zygote keeps (one per GPU slot, at most
        8; ``ZYGOTE_EMBRYOS`` overrides, 0 = fork on request): a spawn then
        hands its request to a process that already exists instead of
        waiting for two forks of a torch-sized image (profiles/r5_boot)."""
        override = os.environ.get('ZYGOTE_EMBRYOS', '')
        if override.strip():
            return max(0, int(override))
        return min(8, max(1, len(self.slots)))

    def zygote_rocr_embryos(self, template):
        """How many embryos initialise ROCr while they wait (HIP workers
        only; ``ZYGOTE_ROCR_EMBRYOS`` overrides, 0 = none): one per GPU
        device (at most the embryo count), each bound to that GPU
        (``ROCR_VISIBLE_DEVICES=<gpu>`` for its ``hsa_init``), so it opens
        that device alone -- not every device of the node -- and a worker of
        that slot keeps the init.  Each halves a woken standby's boot (~105
        -> ~56 ms, profiles/r5_boot) and takes ROCr's init variance
        (110-300 ms spikes) off the scale-up path, on every slot of an
        8-GPU node (round 5 kept them to managers of one
        or two slots because an unbound embryo opened every device)."""
        if template is None or template.backend not in ('hip', 'auto') or \
                not any(getattr(slot, 'kind', 'gpu') != 'cpu'
                        for slot in self.slots):
            return 0
        override = os.environ.get('ZYGOTE_ROCR_EMBRYOS', '')
        if override.strip():
            wanted = max(0, int(override))
        else:
            # one per device: slots that share a device (a one-GPU
            # rehearsal of eight slots) share its embryo, so the device's
            # process count stays within its budget (16 on the pool)
            wanted = len(self._distinct_gpus())
        return min(self.zygote_embryos(), wanted, len(self._distinct_gpus()))

    def _distinct_gpus(self):
        """The managed GPU slots' devices, first occurrence order."""
        out = []
        for slot in self.slots:
            if getattr(slot, 'kind', 'gpu') == 'gpu' and \
                    slot.visible_id not in out:
                out.append(slot.visible_id)
        return out

    def _check_zygote(self):
        """False (and the zygote forgotten, restarted after a pause) once
        the zygote process has exited."""
        z = self.zygote
        if z is None:
            return False
        if z.alive():
            return True
        logger.warning('Worker zygote %d exited; spawning directly until it '
                       'is restarted.', z.pid)
        self.events.emit('zygote_exit', pid=z.pid, code=z.popen.returncode)
        z.close()
        self.zygote = None
        self._zygote_restart_at = time.monotonic() + 10.0
        return False

    def _retire_zygote(self, reason):
        """A zygote that lost a fork request is not trusted again: killed,
        and restarted after the usual pause."""
        z, self.zygote = self.zygote, None
        if z is None:
            return
        logger.error('Retiring worker zygote %d: %s', z.pid, reason)
        self.events.emit('zygote_retired', pid=z.pid, reason=reason)
        try:
            z.popen.kill()
        except OSError:
            pass
        z.close()
        self._zygote_restart_at = time.monotonic() + 10.0

    def _zygote_for(self, template):
        z = self.zygote
        tpl = self.pool_template
        if z is None or tpl is None:
            return None
        if not self._check_zygote():
            return None
        if not z.poll_ready():
            return None      # still importing: this spawn takes the slow path
        if (template.module != tpl.module or
                template.backend != tpl.backend or
                bare_worker(template) != bare_worker(tpl) or
                any(template.env.get(k) != tpl.env.get(k)
                    for k in self._IMPORT_ENV)):
            return None
        return z

    def _spawn(self, template, role, assign=None, slot=None):
        # a boot is timed from the request, the zygote's fork included
        # (~15 ms for a process that imported torch): what the wake lead
        # must cover
        t_request = time.monotonic_ns()
        cmd_r, cmd_w = os.pipe()
        ev_r, ev_w = os.pipe()
        args = ['--cmd-fd', str(cmd_r), '--ev-fd', str(ev_w),
                '--backend', template.backend]
        # a standby spawned by an arrival wake: the scale-up for the key is
        # due within a tick, so it builds the engine now, not at the assign
        woken = (assign is None and slot is not None and role == 'standby'
                 and time.monotonic() < self._wake_until)
        # every device-mode standby builds its engine at boot, before its
        # node agent joins a generation: the assignment's READY is then the
        # warm-start graph alone, which RCCL's one-time load (seconds, on
        # the agent's thread) cannot hold up (profiles/r4_collision)
        prebuild = woken or (assign is None and slot is not None and
                             role == 'standby' and
                             self.pool_mode == 'device')
        if assign is not None:
            args += ['--assign', json.dumps(assign)]
        elif slot is not None:
            pin = {'gpu': slot.visible_id, 'slot': slot.index,
                   'cpus': slot.cpus, 'preinit': self.pool_mode,
                   'node_fence': self.node is not None}
            pin.update(self.pin_fields())
            if prebuild:
                pin['prebuild'] = self._prebuild_spec(template)
            args += ['--pin', json.dumps(pin)]
        env = self._environment(template)
        popen = None
        via = 'exec'
        try:
            zygote = self._zygote_for(template)
            if zygote is not None:
                try:
                    popen = zygote.fork(args, env, (cmd_r, ev_w))
                    via = 'zygote'
                except (OSError, ValueError) as err:
                    from ..worker.zygote import ZygoteLost
                    logger.warning('zygote fork failed (%s); spawning '
                                   'directly.', err)
                    if isinstance(err, ZygoteLost):
                        # the zygote may still fork a worker on these pipe
                        # ends: retire it and spawn on a fresh pair (the
                        # late worker sees EOF on its command pipe and
                        # exits without an assignment)
                        self._retire_zygote(str(err))
                        os.close(cmd_w)
                        os.close(ev_r)
                        os.close(cmd_r)
                        os.close(ev_w)
                        cmd_r, cmd_w = os.pipe()
                        ev_r, ev_w = os.pipe()
                        args[1], args[3] = str(cmd_r), str(ev_w)
            if popen is None:
                argv = self._interpreter(template) + ['-m', template.module]
                popen = subprocess.Popen(argv + args, env=env,
                                         pass_fds=(cmd_r, ev_w),
                                         close_fds=True,
                                         start_new_session=True)
        finally:
            os.close(cmd_r)
            os.close(ev_w)
        proc = ManagedProcess(popen, Pipe(cmd_w, ev_r), role)
        proc.t_spawn = t_request
        proc.woken = woken
        proc.slot = slot.index if slot is not None else None
        proc.via = via
        proc.pin_mode = getattr(self, 'pin_mode', 'isolate')
        self.events.emit('process_spawn', role=role, pid=popen.pid,
                         slot=proc.slot, via=via,
                         embryo=bool(getattr(popen, 'embryo', False)),
                         request_ms=round((time.monotonic_ns() - t_request)
                                          / 1e6, 3))
        return proc

    def _refill_pool(self):
        """Keep one standby pinned to each of the lowest ``pool_size`` free
        GPUs (the slots the next scale-up will take)."""
        if not self.pool_size or self.pool_template is None or \
                self._stopping:
            return
        changed = False
        if self._reap_standbys():
            changed = True
        if self._park_pool():
            changed = True
        if self.pool_parked:
            if changed:
                self._publish_pool()
            return
        have = len(self.standbys)
        free = self._free_slots()[:self.pool_size]
        now = time.monotonic()
        target = self._standby_target(now, have, len(free))
        if have > target and self._retire_excess(have - target):
            changed = True
            have = len(self.standbys)
        if target > have and not self._spawn_due(now):
            target = have      # spawned one boot time before the tick
        for slot in free:
            if have >= target:
                break
            if slot.index not in self.standbys:
                self.standbys[slot.index] = self._spawn(
                    self.pool_template, 'standby', slot=slot)
                have += 1
                changed = True
        if changed:
            self._publish_pool()

    def _standby_target(self, now, have=0, room=None):
        """How many standbys the pool keeps.  A resident pool
        (``POOL_IDLE_RELEASE_S=0``): ``pool_size``, one per free slot.  A
        deep-idle pool that is awake: one per KEYS_PER_POD keys waiting in
        the managed queues beyond what idle workers will pull -- the
        scale-ups the next tick can make -- and at least one while an
        arrival's wake is held for its tick.  Standbys
        the first tick would not assign would otherwise hold their GPU
        (context, prebuilt engine) through the whole burst; later waiting
        keys get theirs ahead of the tick that scales for them, and a
        drained worker stays as a standby until the park.  At N = 1 nothing
        changes: the one slot is the worker's."""
        if not self.pool_sized_to_demand():
            # resident, or the boot pool (every slot's device verified,
            # then parked)
            return self.pool_size
        kpp = min([max(1, int(r.template.keys_per_pod or 1))
                   for r in self.resources.values()] or [1])
        # workers that will pull a waiting key themselves: running and not
        # busy (a starting one included), not draining
        idle = sum(1 for r in self.resources.values()
                   for w in r.workers.values()
                   if w.state not in (EXITED, DRAINING) and not w.busy)

        cap = self.pool_size if room is None else min(self.pool_size, room)

        def need():
            n = max(0, self._workers_for_waiting(now, kpp) - idle)
            if now < self._wake_until:
                n = max(n, 1)
            return min(cap, n)
        target = need()
        if target > have:
            # a spawn on a reading taken before a worker pulled its key
            # (its ``busy`` is what called us) would overshoot: re-read
            self._next_waiting_check = 0.0
            target = need()
        return target

    def _spawn_due(self, now):
        """Whether a standby for waiting keys is spawned now.  An awake
        pool sized to demand spawns it one wake lead before the tick that
        can assign it, like the arrival wake of a parked pool: spawned at
        once, it would hold its GPU (context, prebuilt engine) unassigned
        for the rest of the tick phase -- 2.5 s on average, 163 GPU-s at
        config 3 under strict (profiles/r5_config3).  ``_spawn_at`` is when
        it becomes due (the manager's loop wakes for it)."""
        self._spawn_at = None
        if not self.pool_sized_to_demand() or self._next_tick is None or \
                now < self._wake_until:
            return True
        lead = self.wake_lead()
        due = self._next_tick - lead
        if now >= due or self._next_tick <= now:
            return True
        self._spawn_at = due
        return False

    def _retire_excess(self, excess, now=None):
        """A pool sized to demand retires standbys it holds beyond its
        target -- typically drained workers recycled mid-burst (a strict
        policy's scale-down), which would otherwise hold their GPU
        (context, engine) until the burst ends -- once they have waited one
        boot time unassigned (the wake lead): a standby the demand comes
        back for later is re-spawned, prebuilt, in that time, so holding
        it any longer only holds its GPU (the former
        tick-long hold kept 387 GPU-s of standbys at config 3 under
        strict).  Oldest-idle first; True if any was retired."""
        if not self.pool_sized_to_demand() or excess <= 0:
            return False
        now = time.monotonic() if now is None else now
        lead = self.wake_lead() if self._wake_boots else \
            self.pool_wake_lead_s
        hold = max(lead, self.pool_idle_release_s)
        if self._next_tick is not None and self._next_tick - now > lead and \
                now >= self._wake_until:
            # the next tick that could assign it is further away than a
            # boot: a standby it needs is spawned one lead before it
            # (``_spawn_due``), so nothing is gained by holding this one
            hold = self.pool_idle_release_s
        idle = sorted((proc.standby_since, index)
                      for index, proc in self.standbys.items()
                      if proc.booted and proc.standby_since is not None and
                      now - proc.standby_since > hold)
        retired = 0
        for _, index in idle[:excess]:
            proc = self.standbys.pop(index)
            if proc.popen.poll() is None:
                proc.pipe.send({'cmd': 'exit'})
                self.retiring.append(proc)
            retired += 1
        if retired:
            self.events.emit('standby_retired', standbys=retired,
                             reason='beyond demand')
        return retired > 0

    def pool_sized_to_demand(self):
        """The pool leaves slots empty on purpose (deep idle after the boot
        pool parked): the node communicator spans the slots that have a
        process instead of waiting for all of them."""
        return self.pool_idle_release_s > 0 and self.pool_parks > 0

    def _waiting_keys(self, now):
        """Keys waiting in the managed queues (one pipelined LLEN per queue,
        at most every ``pool_wake_poll_s``; the last reading in between)."""
        if now >= self._next_waiting_check:
            self._next_waiting_check = now + max(self.pool_wake_poll_s, 0.02)
            lengths = self._queue_lengths()
            if lengths is not None:
                self._waiting = sum(lengths.values())
                self._waiting_by_queue = lengths
        return self._waiting

    def _workers_for_waiting(self, now, kpp):
        """Workers the keys waiting now justify: ceil(keys / KEYS_PER_POD)
        in all, or, under the reference policy (``wake_policy``), its
        per-queue floor division summed over the managed resources -- the
        keys a reference tick strands below KEYS_PER_POD get no standby."""
        waiting = self._waiting_keys(now)
        by_queue = getattr(self, '_waiting_by_queue', None)
        if self.wake_policy != 'reference' or not by_queue or \
                not self.resources:
            return -(-waiting // kpp)
        # each queue once (resources of several autoscalers may share one),
        # at the smallest KEYS_PER_POD that reads it
        queue_kpp = {}
        for r in self.resources.values():
            for q in r.template.queues:
                k = max(1, int(r.template.keys_per_pod or 1))
                queue_kpp[q] = min(k, queue_kpp.get(q, k))
        return sum(by_queue.get(q, 0) // k for q, k in queue_kpp.items())

    def _queue_lengths(self):
        """``{queue: LLEN}`` over every managed queue, or None."""
        if self.redis is None:
            return None
        queues = sorted(set(q for r in self.resources.values()
                            for q in r.template.queues))
        if not queues:
            return {}
        self.queue_reads += len(queues)
        try:
            pipe = self.redis.pipeline(transaction=False)
            for queue in queues:
                pipe.llen(queue)
            return dict(zip(queues, (int(n or 0) for n in pipe.execute())))
        except Exception as err:  # pylint: disable=broad-except
            logger.debug('queue length check failed: %s', err)
            return None

    def _park_pool(self):
        """Deep idle (``POOL_IDLE_RELEASE_S``): with no declared or live
        worker for that long, retire every standby -- the node then holds
        no GPU, like the reference at zero replicas -- and keep the pool
        empty until demand returns: a key's arrival (``pool_wake_poll_s``,
        woken ``wake_lead()`` before the next tick) or, without it, the
        scale-up itself, which is then a cold spawn with the pool refilling
        behind it.  True if standbys were retired."""
        now = time.monotonic()
        self._park_at = None
        demand = any(r.declared > 0 or any(w.state != EXITED
                                           for w in r.workers.values())
                     for r in self.resources.values())
        self._arrival_watch = not demand
        if demand:
            self._last_demand = now
            self._queued = {}
            self._wake_at = None
            self._wake_until = 0.0    # the tick scaled: the hold is done
            if self.pool_parked:
                self.pool_parked = False
                self.events.emit('pool_resumed',
                                 queue_reads=self.queue_reads,
                                 queue_reads_fine=self.queue_reads_fine)
                logger.info('Demand returned: refilling the warm pool.')
            return False
        released = [p for p in self.standbys.values()
                    if p.booted and not p.engine_cached and
                    self.pool_mode == 'device']
        arrived = (self.pool_idle_release_s > 0 or bool(released)) and \
            self._arrived(now)
        if arrived and released:
            # ENGINE_IDLE_RELEASE_S freed these standbys' engines: a key's
            # arrival has them rebuild it before the scale-up tick
            for proc in released:
                proc.pipe.send({'cmd': 'prebuild',
                                'spec': self._prebuild_spec(
                                    self.pool_template)})
                proc.engine_cached = True     # (until told otherwise)
            self.events.emit('engine_rebuild', standbys=len(released))
        if arrived and self.pool_idle_release_s > 0:
            wake_at = now
            lead = self.wake_lead()
            if self.pool_parked and lead > 0 and \
                    self._next_tick is not None and \
                    self._next_tick - now > lead:
                wake_at = self._next_tick - lead
            if self._wake_at is None or wake_at < self._wake_at:
                self._wake_at = wake_at
        if self._wake_at is not None and now >= self._wake_at:
            self._wake_at = None
            if self.pool_parked and not self._tick_would_scale():
                # KEYS_PER_POD: the reference's floor division does not
                # scale for these keys; a standby woken for them would hold
                # its GPU (context, prebuilt engine) for the whole wake
                # hold.  The next arrival re-arms the wake.
                self.wake_deferrals += 1
                self.events.emit('wake_deferred', waiting=self._waiting,
                                 policy=self.wake_policy)
                return False
            self._last_demand = now
            self._wake_until = now + self.pool_wake_hold_s
            if self.pool_parked:
                self.pool_parked = False
                self.arrival_wakes += 1
                self.events.emit('pool_resumed', reason='arrival',
                                 queue_reads=self.queue_reads,
                                 queue_reads_fine=self.queue_reads_fine,
                                 lead_s=round(self.wake_lead(), 4),
                                 tick_in_s=(round(self._next_tick - now, 4)
                                            if self._next_tick is not None
                                            else None))
                logger.info('Keys arrived: refilling the warm pool ahead of '
                            'the scale-up tick.')
            return False
        if self.pool_idle_release_s <= 0 or self.pool_parked:
            return False
        if now - self._last_demand < self.pool_idle_release_s or \
                now < self._wake_until:
            # the loop wakes for it (0.01 s after demand ends, by default)
            # instead of at its next queue read
            self._park_at = max(self._last_demand + self.pool_idle_release_s,
                                self._wake_until)
            return False
        self.pool_parked = True
        self.pool_parks += 1
        released = 0
        for index, proc in list(self.standbys.items()):
            if proc.popen.poll() is None:
                proc.pipe.send({'cmd': 'exit'})
                self.retiring.append(proc)
                released += 1
            del self.standbys[index]
        self.events.emit('pool_parked', standbys=released,
                         idle_s=round(now - self._last_demand, 3),
                         queue_reads=self.queue_reads,
                         queue_reads_fine=self.queue_reads_fine)
        logger.info('No demand for %.0f s: released %d standby process(es).',
                    now - self._last_demand, released)
        return True

    def note_next_tick(self, t_monotonic):
        """The autoscaler loop's next tick instant (``time.monotonic``
        seconds, system-wide, so a ``unix:`` daemon's clients report it
        too): a deferred arrival wake is timed against it.  With several
        autoscalers on one manager the earliest upcoming tick wins (a
        report replaces a tick that is due or past).  Called from the
        loop's thread: under the manager lock."""
        t_monotonic = float(t_monotonic)
        with self.lock:
            current = self._next_tick
            if current is None or current <= time.monotonic() + 0.05 or \
                    t_monotonic < current:
                self._next_tick = t_monotonic
            lead = self.wake_lead()
            if self._wake_at is not None and lead > 0:
                # the tick came earlier than planned for (IDLE_INTERVAL)
                self._wake_at = min(self._wake_at, self._next_tick - lead)
        self._wake()

    # margin of the wake lead over the boot it is sized for, from the
    # measured spread (not constants fitted on one box):
    # FLOOR covers the spawn request (0.5 ms from an embryo) and the loop's
    # wake-up; SPREAD_K times the distance between the sized boot and the
    # median boot covers the jitter the recent boots show, so a busier
    # 8-GPU host with concurrent boots gets a wider margin by itself.
    # Replayed (tools/wake_lead_replay.py) over round 5's 576 woken boots
    # without ROCr embryos: late 5.1 ms / hold 79 ms a wake against 3.9 / 83
    # for the former fixed +50 ms; over the ROCr-embryo boots (round 5: 50,
    # round 6: 24) never late, hold 22-26 ms a wake against 32 for the
    # former fixed +30 ms.  K = 3 held 7 ms a wake more on round 6's boots
    WAKE_MARGIN_FLOOR_S = 0.01
    WAKE_SPREAD_K = 1.5
    WAKE_MARGIN_MAX_S = 0.06
    # (while fewer than 4 boots are known: the slowest plus this)
    WAKE_MARGIN_S = 0.05

    def wake_margin(self, boots=None):
        """Seconds of lead beyond the sized boot (see the constants)."""
        boots = sorted(self._wake_boots if boots is None else boots)
        if len(boots) < 4:
            return self.WAKE_MARGIN_S
        sized, median = boots[-2], boots[len(boots) // 2]
        return min(self.WAKE_MARGIN_MAX_S,
                   max(self.WAKE_MARGIN_FLOOR_S,
                       self.WAKE_MARGIN_FLOOR_S +
                       self.WAKE_SPREAD_K * (sized - median)))

    def wake_lead(self):
        """Seconds before the next tick an arrival wakes a parked pool:
        ``pool_wake_lead_s`` until woken standbys have been timed, then the
        second slowest of the last 16 spawn -> booted+prebuilt times (the
        slowest while fewer than 4 are known) plus :meth:`wake_margin`,
        never above ``pool_wake_lead_s``.  Every second of lead beyond the
        boot is a standby holding its GPU unassigned; a boot slower than
        the lead is late by the difference.  The boot's spread is the HIP
        context (50-70 ms, now and then 150 ms, once in a while 0.5 s:
        profiles/r4_boot, profiles/r5_boot), so the slowest sample is an
        outlier the next wakes rarely repeat: over 576 woken boots of rounds
        4-5, the second slowest of 16 is late less often and by less than
        the slowest of 8 and holds less (tools/wake_lead_replay.py)."""
        cap = self.pool_wake_lead_s
        if cap <= 0 or not self._wake_boots:
            return cap
        boots = sorted(self._wake_boots)
        sized = boots[-2] if len(boots) >= 4 else boots[-1]
        return min(cap, sized + self.wake_margin(boots))

    def _prebuild_spec(self, template):
        """What an arrival-woken standby builds its engine for: the shape
        (kind, keys per pod) of the resource its template serves."""
        for resource in self.resources.values():
            if resource.template.module == template.module:
                return {'kind': resource.kind,
                        'keys_per_pod': resource.template.keys_per_pod}
        return {'kind': 'deployment', 'keys_per_pod': template.keys_per_pod}

    def _arrival_check_due(self):
        """When the next queue-length read is due while arrivals are
        watched (else None): the manager's loop must not sleep past it --
        its idle timeout (50 ms) was the real poll period, so a key was
        seen up to 50 ms late instead of ``pool_wake_poll_s``
        (profiles/r5_boot)."""
        if not self._arrival_watch or not self._arrival_reads():
            return None
        return self._next_arrival_check

    def _arrival_reads(self):
        """Whether ``_park_pool`` reads the queues for arrivals on this
        pass: a deep-idle pool, or standbys whose engines were released.  A
        resident pool (``POOL_IDLE_RELEASE_S=0``) never does, so its loop
        must not wake for a read that is never taken (a stale
        ``_next_arrival_check`` made the loop spin at 1 kHz)."""
        if self.pool_wake_poll_s <= 0 or self.redis is None:
            return False
        if self.pool_idle_release_s > 0:
            return True
        return self.pool_mode == 'device' and any(
            p.booted and not p.engine_cached for p in self.standbys.values())

    # queue-read period inside the wake window (the last ``wake_lead()``
    # before a parked pool's tick): an arrival there wakes the pool at once,
    # so each ms it goes unseen is a ms of the standby's boot lost
    ARRIVAL_FINE_S = 0.004
    # queue-read period of a parked pool outside the wake window while the
    # next tick is known: a key seen there is woken at the window's start
    # anyway, so the reads only have to land before it.  10 reads/s per
    # queue instead of 50 (the reference reads twice per INTERVAL,
    # autoscaler.py:64-71); the window's first read is never skipped
    ARRIVAL_FAR_S = 0.1

    def _next_arrival_read(self, now):
        """``pool_wake_poll_s`` after ``now``, but never past the start of
        the next tick's wake window, and ``ARRIVAL_FINE_S`` inside it: a key
        seen before the window is woken at the window's start anyway, one
        seen inside it is woken on sight."""
        period = self.pool_wake_poll_s
        if self._next_tick is None or not self.pool_parked:
            return now + period
        window = self._next_tick - self.wake_lead()
        if now >= window:
            if now >= self._next_tick:
                return now + period
            return now + min(period, self.ARRIVAL_FINE_S)
        return min(now + max(period, self.ARRIVAL_FAR_S), window)

    def _arrived(self, now):
        """True when a managed queue grew since the last check (read every
        ``pool_wake_poll_s`` while no worker is declared or live).  Growth,
        not length: keys a policy strands below KEYS_PER_POD do not hold
        the pool, new ones wake it.  One pipelined LLEN per queue."""
        if self.pool_wake_poll_s <= 0 or self.redis is None or \
                now < self._next_arrival_check:
            return False
        self._next_arrival_check = self._next_arrival_read(now)
        if self.pool_parked and self._next_tick is not None and \
                self._next_tick - self.wake_lead() <= now < self._next_tick:
            self.queue_reads_fine += len(set(
                q for r in self.resources.values() for q in r.template.queues))
        lengths = self._queue_lengths()
        if not lengths:
            return False
        queues = sorted(lengths)
        self._waiting = sum(lengths.values())
        self._waiting_by_queue = lengths
        self._next_waiting_check = now + self.pool_wake_poll_s
        before, self._queued = self._queued, lengths
        grown = [q for q in queues if lengths[q] > before.get(q, 0)]
        if grown:
            self.events.emit('arrival', queues=grown,
                             parked=self.pool_parked)
        return bool(grown)

    def _tick_would_scale(self):
        """Whether the next tick scales up for the keys waiting now: the
        autoscaler's policy (``wake_policy``) from zero replicas, per managed
        resource over its queues and KEYS_PER_POD.  Under ``reference`` one
        key below KEYS_PER_POD scales nothing (floor division per queue,
        ``/root/reference/autoscaler/autoscaler.py:217``); under ``strict``
        any key does.  True without a known policy or a reading (wake, as
        before).  One pipelined LLEN per queue."""
        if self.wake_policy not in policy.POLICIES or not self.resources:
            return True
        lengths = self._queue_lengths()
        if lengths is None:
            return True
        self._waiting = sum(lengths.values())
        self._waiting_by_queue = lengths
        for resource in self.resources.values():
            keys = {q: lengths.get(q, 0) for q in resource.template.queues}
            kpp = max(1, int(resource.template.keys_per_pod or 1))
            if policy.decide(keys, 0, 1 << 30, kpp, 0,
                             policy=self.wake_policy) > 0:
                return True
        return False

    def _take_standby(self, template, slot):
        """The standby pinned to ``slot`` (booted or still booting: it
        reads the assignment as soon as its imports finish)."""
        if self.pool_template is None or \
                template.module != self.pool_template.module or \
                template.backend != self.pool_template.backend:
            return None
        proc = self.standbys.get(slot.index)
        if proc is None or proc.popen.poll() is not None:
            return None
        if getattr(proc, 'pin_mode', 'isolate') != \
                getattr(self, 'pin_mode', 'isolate'):
            return None      # pinned the old way (WORKER_PIN=auto switched)
        del self.standbys[slot.index]
        self._publish_pool()
        return proc

    def _publish_slots(self):
        """The slot table as verified so far (``kiosk:slots``): the bench
        samples amdsmi on these PCI addresses, not on KFD order."""
        if self.redis is None:
            return
        try:
            self.redis.set(SLOTS_KEY, json.dumps([
                {'index': s.index, 'visible': s.visible_id, 'pci': s.pci,
                 'verified': bool(getattr(s, 'pci_verified', False)),
                 'kind': s.kind} for s in self.slots]))
        except Exception:  # pylint: disable=broad-except
            pass

    def _publish_pool(self):
        if self.redis is None:
            return
        try:
            # booted standbys, standbys, node communicator state, parked
            # (POOL_IDLE_RELEASE_S: the pool is empty on purpose)
            self.redis.set(POOL_KEY, '%d %d %s %d' % (
                sum(1 for p in self.standbys.values() if p.booted),
                len(self.standbys),
                self.node.state if self.node is not None else 'off',
                int(self.pool_parked)))
        except Exception:  # pylint: disable=broad-except
            pass

    def _on_standby_messages(self, proc):
        for message in proc.pipe.read_messages():
            if message is None:
                proc.eof = True
                continue
            self._on_standby_message(proc, message)

    def _on_standby_message(self, proc, message):
        if self.node is not None and message.get('ev') in NODE_EVENTS:
            self.node.on_message(proc, message)
            return
        if any(p is proc for p in self.retiring):
            # a process retired on its 'recycled' report still sends the
            # 'standby' of its recycle in the same batch: it is no standby
            return
        if message.get('ev') == 'engine_released':
            proc.engine_cached = False
            proc.hbm_free = message.get('hbm_free')
            self.events.emit('engine_released', pid=proc.pid, slot=proc.slot,
                             released_bytes=message.get('released_bytes'),
                             hbm_free=proc.hbm_free)
            return
        if message.get('ev') == 'device':
            self._check_device(proc, message.get('pci'))
            return
        if message.get('ev') == 'prebuilt':
            proc.engine_cached = not message.get('error')
            self.events.emit('standby_prebuilt', pid=proc.pid, slot=proc.slot,
                             ms=message.get('ms'),
                             hbm_bytes=message.get('hbm_bytes'),
                             stages=message.get('stages'),
                             error=message.get('error'))
            return
        if message.get('ev') == 'standby':
            proc.engine_cached = bool(message.get('engine_cached'))
            if proc.woken and not proc.booted:
                # spawn -> booted and prebuilt: what the wake lead must cover
                # (once: a recycled worker reports 'standby' again later)
                proc.woken = False
                self._wake_boots.append(
                    (time.monotonic_ns() - proc.t_spawn) / 1e9)
            proc.booted = True
            proc.standby_since = time.monotonic()
            proc.hbm_free = message.get('hbm_free')
            if message.get('pci'):
                if not self._check_device(proc, message.get('pci')):
                    return   # retired: the pool respawns it re-pinned
            self._publish_pool()
            self.events.emit('standby_ready', pid=proc.pid, slot=proc.slot,
                             boot_s=(time.monotonic_ns() - proc.t_spawn)
                             / 1e9, preinit=message.get('preinit'),
                             recycled=proc.role == 'standby' and
                             proc.recycles > 0)

    def _check_device(self, proc, pci):
        """the slot table maps slot -> HIP ordinal -> PCI address
        from KFD topology order, which drives the HIP_VISIBLE_DEVICES pin,
        the NUMA-local CPU affinity and the BDF the benchmark's amdsmi
        cross-check samples.  The process reports the PCI address HIP sees
        for its ordinal; on a mismatch the slot is remapped to the device
        actually behind that ordinal (its NUMA node and CPUs re-read) and a
        standby pinned with the wrong affinity is respawned.  False when
        ``proc`` was retired for that."""
        from .gpus import local_cpus, normalize_pci
        index = proc.slot
        slot = next((s for s in self.slots if s.index == index), None)
        actual = normalize_pci(pci)
        if slot is None or slot.kind != 'gpu' or actual is None:
            return True
        expected = normalize_pci(slot.pci)
        proc.pci = actual
        if expected == actual:
            if not getattr(slot, 'pci_verified', False):
                slot.pci_verified = True
                self.events.emit('gpu_mapping', slot=index, pci=actual,
                                 visible=slot.visible_id, verified=True)
                self._publish_slots()
            return True
        slot.pci = actual
        slot.numa_node, slot.cpus = local_cpus(actual)
        slot.pci_verified = True
        self.mapping_fixes += 1
        self.events.emit('gpu_mapping_mismatch', slot=index,
                         visible=slot.visible_id, expected=expected,
                         actual=actual, numa_node=slot.numa_node)
        logger.error('GPU slot %d (HIP_VISIBLE_DEVICES=%s) is %s, not %s as '
                     'KFD order suggested: remapped (NUMA node %s).', index,
                     slot.visible_id, actual, expected, slot.numa_node)
        self._publish_slots()
        if self.standbys.get(index) is proc and expected is not None:
            del self.standbys[index]
            proc.pipe.send({'cmd': 'exit'})
            self.retiring.append(proc)
            return False
        return True

    def _recycle_ok(self, resource):
        tpl = self.pool_template
        return bool(self.recycle and self.pool_size and tpl is not None and
                    not self._stopping and
                    resource.template.module == tpl.module and
                    resource.template.backend == tpl.backend)

    def _on_recycled(self, worker, message):
        """A worker finished cleanly and kept its process: account for it
        like an exit, then adopt the process as its GPU's standby."""
        if worker.state == EXITED:
            return
        resource = worker.resource
        proc = worker.proc
        self._on_exit(resource, worker, int(message.get('code', 0)),
                      recycled=True)
        slot = worker.slot
        proc.recycles += 1
        if (self._recycle_ok(resource) and slot.index not in self.standbys
                and len(self.standbys) < self.pool_size and
                not self._parks_on_recycle() and
                getattr(proc, 'pin_mode', 'isolate') ==
                getattr(self, 'pin_mode', 'isolate') and
                not getattr(proc, 'node_quarantined', False)):
            proc.role = 'standby'
            proc.slot = slot.index
            proc.booted = False     # until its 'standby' message
            self.standbys[slot.index] = proc
            self._publish_pool()
            self.events.emit('worker_recycled', worker=worker.id,
                             gpu=slot.index, pid=proc.pid)
        else:
            proc.pipe.send({'cmd': 'exit'})
            self.retiring.append(proc)
            # its GPU is held until the process is gone (standby_exit)
            self.events.emit('worker_retired', worker=worker.id,
                             gpu=slot.index, pid=proc.pid)

    # a release delay this short is the deep-idle default (0.01 s): the
    # drained worker would be parked before anything could assign it
    PARK_AT_ONCE_S = 0.05

    def _parks_on_recycle(self):
        """A drained worker comes back when deep idle would park the pool
        on this very pass (no resource declares or runs a worker, no
        arrival's wake is held): it is retired at once instead of kept as a
        standby for ``POOL_IDLE_RELEASE_S`` first -- its exit starts ~10 ms
        earlier on every wake (standby time)."""
        if not 0 < self.pool_idle_release_s <= self.PARK_AT_ONCE_S or \
                time.monotonic() < self._wake_until:
            return False
        return not any(r.declared > 0 or any(w.state != EXITED
                                             for w in r.workers.values())
                       for r in self.resources.values())

    ORPHAN_SCAN_S = 5.0

    def _reap_orphans(self, now=None):
        """Subreaper hygiene: a descendant a worker orphaned is
        re-parented to this process; nothing waits for it, so it would stay
        a zombie for the daemon's life.  Every ``ORPHAN_SCAN_S`` the direct
        children in state Z that are none of ours are reaped -- by pid, and
        only after a zombie was seen on two scans (an embedding program's
        own ``subprocess`` children are reaped by their owner well before
        that), never with a blind ``waitpid(-1)``."""
        now = time.monotonic() if now is None else now
        if now < getattr(self, '_orphan_scan_at', 0.0):
            return []
        self._orphan_scan_at = now + self.ORPHAN_SCAN_S
        if not self.zygote_enabled:
            return []     # not a subreaper: orphans go to init
        me = os.getpid()
        ours = set(p.pid for p in self.standbys.values())
        ours.update(p.pid for p in self.retiring)
        ours.update(w.proc.pid for r in self.resources.values()
                    for w in r.workers.values())
        if self.zygote is not None:
            ours.add(self.zygote.pid)
        seen = getattr(self, '_zombies_seen', set())
        zombies = set()
        try:
            names = os.listdir('/proc')
        except OSError:
            return []
        for name in names:
            if not name.isdigit() or int(name) in ours:
                continue
            try:
                with open('/proc/%s/stat' % name) as f:
                    stat = f.read()
            except OSError:
                continue
            fields = stat[stat.rfind(')') + 2:].split()
            if len(fields) > 1 and fields[0] == 'Z' and int(fields[1]) == me:
                zombies.add(int(name))
        reaped = []
        for pid in zombies & seen:
            try:
                if os.waitpid(pid, os.WNOHANG)[0] == pid:
                    reaped.append(pid)
            except ChildProcessError:
                pass
        self._zombies_seen = zombies - set(reaped)
        if reaped:
            self.events.emit('orphans_reaped', pids=reaped)
        return reaped

    def _reap_standbys(self):
        """Forget exited standby / retired processes (``standby_exit``
        closes their standby GPU time in the metrics).  True if a retired
        process was reaped."""
        retired = False
        for index, proc in list(self.standbys.items()):
            if proc.popen.poll() is not None:
                proc.close()
                del self.standbys[index]
                self.events.emit('standby_exit', pid=proc.pid, slot=index,
                                 code=proc.popen.returncode)
        for proc in list(self.retiring):
            if proc.popen.poll() is not None:
                exiting = self._exiting_t(proc)
                proc.close()
                self.retiring.remove(proc)
                self.events.emit('standby_exit', pid=proc.pid, slot=proc.slot,
                                 code=proc.popen.returncode, retired=True,
                                 exiting_t=exiting)
                retired = True
        return retired

    @staticmethod
    def _exiting_t(proc):
        """When a retired process called ``os._exit`` (its last message,
        ``exiting``): the rest of its exit is the kernel's teardown."""
        t = None
        try:
            for message in proc.pipe.read_messages():
                if message is not None and message.get('ev') == 'exiting':
                    t = message.get('t')
        except (OSError, AttributeError, ValueError):
            return None
        return t
