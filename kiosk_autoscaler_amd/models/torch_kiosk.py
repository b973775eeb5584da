"""PyTorch-ROCm worker engine on the hand-written gfx950 kernels.

``WORKER_ENGINE=kiosk_autoscaler_amd.models.torch_kiosk:TorchKioskEngine``
runs the worker model (``MODEL_LAYERS`` blocks of ``MODEL_DIM`` ->
``MODEL_HIDDEN`` -> ``MODEL_DIM``, tanh-GELU, residual, bf16) in a PyTorch
process, with every byte of device memory a torch tensor (torch's caching
allocator, torch's stream) and every kernel one of ours:

* weights: bf16 / fp32 torch tensors filled by the N2 init kernel with the
  built-in engine's seeds (:func:`~..ops.kernels.model_weights`), so both
  engines serve bit-identical outputs for the same job;
* forward: per layer the 256x256 LDS-ring GEMM with the fused bias+GELU
  epilogue, then the down-projection GEMM with the fused bias+residual
  epilogue (split-K into a preallocated workspace where the grid alone would
  leave CUs idle), then the deterministic partial-sum kernel -- the whole
  forward, input generation included, captured once into a native hipGraph
  (``StreamGraph``, not ``torch.cuda.CUDAGraph``: no RNG state or memory
  pool to set up on a woken standby's critical path, profiles/r5_boot).
  The job's seed reaches the captured input kernel through a pinned host
  word copied inside the graph, so a forward is exactly one graph launch;
* N1 warm-start: the warm-start kernel over the engine's own first weight
  matrix (every CU, the GEMM's LDS ring zeroed, an MFMA loop), captured as
  a second graph: once the engine is built, READY is one graph launch --
  which RCCL's one-time load on the node agent's thread cannot hold up
  (``profiles/r4_collision``).

The reference's worker is whatever image its Deployment runs
(``/root/reference/autoscaler/autoscaler.py:235-237``); this is the
framework's own PyTorch-ROCm one.
"""
import time

from ..ops import kernels as ops
from ..ops import native

# MFMA iterations of the warm-start loop (the native engine's default)
_WARM_ITERS = 4096


_ALIGN = 256


def _aligned(nbytes):
    return (nbytes + _ALIGN - 1) // _ALIGN * _ALIGN


def _nbytes(shape, dtype):
    import torch
    count = 1
    for d in shape:
        count *= int(d)
    return count * torch.empty((), dtype=dtype).element_size()


def _span(specs):
    return sum(_aligned(_nbytes(shape, dtype)) for _, shape, dtype in specs)


def _layer_bytes(dim, hidden):
    """One layer's w1, b1, w2, b2 as :func:`ops.model_weights` lays them."""
    import torch
    return _span([('w1', (hidden, dim), torch.bfloat16),
                  ('b1', (hidden,), torch.float32),
                  ('w2', (dim, hidden), torch.bfloat16),
                  ('b2', (dim,), torch.float32)])


class _Carver(object):
    """Hands out 256-B aligned typed views of one uint8 device tensor."""

    def __init__(self, arena):
        self.arena = arena
        self.offset = 0

    def __call__(self, shape, dtype):
        n = _nbytes(shape, dtype)
        if self.offset + n > self.arena.numel():
            raise RuntimeError('arena overflow: %d + %d > %d'
                               % (self.offset, n, self.arena.numel()))
        view = self.arena[self.offset:self.offset + n].view(dtype)
        self.offset += _aligned(n)
        return view.view(tuple(int(d) for d in shape))


def _select_device(torch):
    """``WORKER_PIN=visible`` (every managed GPU visible): the worker's own
    GPU is ``KIOSK_DEVICE``; with the default pin it is the only one."""
    from ..worker.pinning import device_ordinal
    ordinal = device_ordinal()
    if ordinal != torch.cuda.current_device():
        torch.cuda.set_device(ordinal)


class TorchKioskEngine(object):
    name = 'torch-kiosk'
    # no collective of its own: the worker caps the node communicator's
    # RCCL channels (worker/main.py; 166 MB of HBM instead of 670 MB)
    collectives = False

    @staticmethod
    def warm_device():
        """Standby boot (``worker/main.py``): torch's lazy CUDA init plus
        our launch handles -- no hipBLASLt handle (this engine never calls
        a torch matmul) and no torch fill: the engine clears its buffers
        with ``hipMemsetAsync`` and captures its graphs natively
        (profiles/r4_comgr, profiles/r5_boot)."""
        import torch
        torch.cuda.init()
        _select_device(torch)
        native.load().prepare_kernels()

    def __init__(self, cfg, stage=None):
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError('TorchKioskEngine needs a GPU')
        self.torch = torch
        self.mod = native.load()       # after torch: one HIP runtime
        _select_device(torch)
        self.device = torch.device('cuda', torch.cuda.current_device())
        self.dim, self.hidden, self.layers = cfg.dim, cfg.hidden, cfg.layers
        self.max_rows = max(int(cfg.rows) * int(cfg.batch), 256)
        self.seed = int(cfg.seed)
        # LDS limits, code objects, launch handles: once, outside capture
        self.mod.prepare_kernels()
        if stage:
            stage('kernels_prepared')
        # the stream the standby's preinit_device warmed (it paid the
        # process's first hardware-queue set-up, ~85 ms in torch's HIP
        # runtime, profiles/r4_boot); handed back on close for the next
        # engine
        self._device_index = torch.cuda.current_device()
        self._stream_handle = self.mod.take_stream(self._device_index)
        if self._stream_handle:
            self.stream = torch.cuda.ExternalStream(self._stream_handle,
                                                    device=self.device)
        else:
            self.stream = torch.cuda.Stream()
        if stage:
            stage('stream_ready')
        rows, dim, hidden = self.max_rows, self.dim, self.hidden
        # the split-K workspace any row count up to the capacity can want
        # (the split count changes at 256-row steps; the built-in engine
        # probes the same rows, so both arenas have one size, utils/hbm.py)
        ws = 0
        for m in range(256, rows + 256, 256):
            m = min(m, rows)
            ws = max(ws, self.mod.gemm_workspace_bytes(m, hidden, dim),
                     self.mod.gemm_workspace_bytes(m, dim, hidden))
        self.workspace_bytes = ws
        f32, i32, i64 = torch.float32, torch.int32, torch.int64
        bf16 = torch.bfloat16
        # one device allocation for everything (as the built-in engine's
        # arena): the small buffers that start zeroed first, so one fill
        # clears them, then the weights and the activations
        small = [('partials', (self.mod.sum_blocks,), f32),
                 ('seed_dev', (1,), i64),
                 ('warm_record', (self._cus() * 8,), i32)]
        big = [('x', (rows, dim), bf16),          # input / ping
               ('y', (rows, dim), bf16),          # pong
               ('h', (rows, hidden), bf16),
               ('workspace', (max(1, ws // 4),), f32)]
        weight_bytes = _layer_bytes(dim, hidden) * self.layers
        total = (_span(small) + weight_bytes + _span(big))
        if stage:
            stage('sized')
        with torch.cuda.stream(self.stream):
            # one hipMalloc by the native module, handed over by DLPack: the
            # arena lives outside torch's caching allocator (no rounding, no
            # cached segment left after close); the tensor frees the buffer
            # when its last view dies
            from torch.utils.dlpack import from_dlpack
            self.arena = from_dlpack(self.mod.device_buffer(
                total, torch.cuda.current_device()))
            if stage:
                stage('arena_allocated')
            carve = _Carver(self.arena)
            for name, shape, dtype in small:
                setattr(self, name, carve(shape, dtype))
            self.mod.memset_async(self.arena.data_ptr(), 0, carve.offset,
                                  self.stream.cuda_stream)
            self.weights = ops.model_weights(dim, hidden, self.layers,
                                             self.seed, alloc=carve)
            for name, shape, dtype in big:
                setattr(self, name, carve(shape, dtype))
        if stage:
            stage('weights_enqueued')
        self.seed_host = torch.zeros(1, dtype=i64).pin_memory()
        # the forward's partial sums land here inside the graph: the key's
        # checksum needs no torch kernel (a kernel launch would wait while
        # RCCL loads on the node agent's thread; a graph launch does not)
        self.partials_host = torch.zeros(self.mod.sum_blocks,
                                         dtype=f32).pin_memory()
        if stage:
            stage('host_pinned')
        self.stream.synchronize()
        if stage:
            stage('weights_on_device')
        self.graphs = {}               # rows -> (StreamGraph, output tensor)
        self.warm_graph = None
        self._capture(self.max_rows)
        if stage:
            stage('forward_captured')
        self._capture_warm()
        if stage:
            stage('graphs_ready')

    # -- construction -----------------------------------------------------
    def _cus(self):
        # one attribute query: torch's get_device_properties costs ~0.1 s
        # on its first call (profiles/r4_boot)
        if not hasattr(self, '_cu_count'):
            self._cu_count = int(self.mod.device_cus(self._device_index))
        return self._cu_count

    def _enqueue_forward(self, rows):
        """The forward on the current stream (captured, never run eagerly
        outside a graph)."""
        mod = self.mod
        stream = self.stream.cuda_stream
        mod.memcpy_async(self.seed_dev.data_ptr(), self.seed_host.data_ptr(),
                         8, stream)
        x = self.x[:rows]
        mod.init_uniform_bf16_devseed(x.data_ptr(), x.numel(),
                                      self.seed_dev.data_ptr(), -1.0, 1.0,
                                      stream)
        cur, nxt = self.x, self.y
        h = self.h[:rows]
        for w1, b1, w2, b2 in self.weights:
            mod.gemm(cur.data_ptr(), w1.data_ptr(), h.data_ptr(),
                     b1.data_ptr(), 0, rows, self.hidden, self.dim,
                     ops.EPILOGUES['gelu'], stream, ops.VARIANTS['auto'],
                     self.workspace.data_ptr(), self.workspace_bytes)
            mod.gemm(h.data_ptr(), w2.data_ptr(), nxt.data_ptr(),
                     b2.data_ptr(), cur.data_ptr(), rows, self.dim,
                     self.hidden, ops.EPILOGUES['residual'], stream,
                     ops.VARIANTS['auto'], self.workspace.data_ptr(),
                     self.workspace_bytes)
            cur, nxt = nxt, cur
        out = cur[:rows]
        mod.partial_sums(out.data_ptr(), out.numel(),
                         self.partials.data_ptr(), stream)
        mod.memcpy_async(self.partials_host.data_ptr(),
                         self.partials.data_ptr(),
                         self.partials.numel() * 4, stream)
        return out

    def _record(self, enqueue):
        """Capture ``enqueue()`` (launches on the engine's stream) as a
        native hipGraph (``_kiosk_hip.StreamGraph``): torch.cuda.CUDAGraph
        would also capture torch's RNG state and open a private memory pool
        -- 10-27 ms on a woken standby's first capture, on its path to READY
        (profiles/r5_boot) -- and this engine needs neither.  Thread-local
        capture (as the built-in engine's): the node agent's thread may
        call HIP meanwhile."""
        graph = self.mod.StreamGraph(self.stream.cuda_stream)
        self.stream.synchronize()
        graph.begin()
        try:
            result = enqueue()
        except BaseException:
            graph.abort()
            raise
        graph.end()
        return graph, result

    def _capture(self, rows):
        self.graphs[rows] = self._record(lambda: self._enqueue_forward(rows))
        return self.graphs[rows]

    def _capture_warm(self):
        w1 = self.weights[0][0]

        def enqueue():
            stream = self.stream.cuda_stream
            self.mod.memset_async(self.warm_record.data_ptr(), 0,
                                  self.warm_record.numel() * 4, stream)
            self.mod.warmstart_raw(
                w1.data_ptr(), w1.numel(), self.warm_record.data_ptr(),
                self._cus(), _WARM_ITERS, self.mod.gemm_ring_lds_bytes,
                stream)
        self.warm_graph = self._record(enqueue)[0]

    # -- plug-in contract ---------------------------------------------------
    def warmstart(self):
        """N1: one graph launch (every CU, LDS ring, MFMA loop)."""
        t0 = time.perf_counter()
        self.warm_graph.launch()
        self.stream.synchronize()
        rec = self.warm_record.view(-1, 8)
        return {'backend': 'torch-kiosk', 'blocks': int(rec.shape[0]),
                'wall_us': (time.perf_counter() - t0) * 1e6,
                'graph': True}

    def forward(self, rows, seed):
        """One forward of ``rows`` rows of the ``seed`` input: a graph
        launch (rows other than the captured capacity get their own graph,
        captured once).  Returns the bf16 output view (valid until the next
        forward)."""
        if not 1 <= rows <= self.max_rows:
            raise ValueError('rows=%d outside [1, %d]' % (rows,
                                                          self.max_rows))
        entry = self.graphs.get(rows) or self._capture(rows)
        # the previous replay may still read the pinned seed word
        self.stream.synchronize()
        self.seed_host[0] = int(seed)
        entry[0].launch()
        return entry[1]

    def infer(self, jobs):
        """One forward per job; ``service_ms`` (the benchmark's fixed
        per-key GPU time) repeats it until that much time has passed."""
        out = []
        for job in jobs:
            t0 = time.perf_counter()
            rows, seed = int(job['rows']), int(job['seed'])
            self.forward(rows, seed)
            passes = 1
            budget = float(job.get('service_ms') or 0) / 1e3
            while True:
                self.stream.synchronize()
                if time.perf_counter() - t0 >= budget:
                    break
                self.forward(rows, seed)
                passes += 1
            out.append({'output_sum': '%.6e' % self.checksum(),
                        'passes': passes, 'engine': self.name})
        return out

    def checksum(self):
        """The last forward's output sum: its per-block partials added in
        block order in double, as the built-in engine does
        (``Engine::forward``, ``csrc/runtime/engine.cpp``).  Call after the
        stream is synchronised."""
        total = 0.0
        for value in self.partials_host.tolist():
            total += value
        return total

    def output(self, rows, seed):
        """The forward's ``[rows, dim]`` output as a fresh tensor (tests)."""
        y = self.forward(rows, seed)
        self.stream.synchronize()
        return y.clone()

    def hbm_bytes(self):
        return int(self.arena.numel()) if self.arena is not None else 0

    def close(self):
        if self.stream is None:
            return
        # nothing of ours may still run when the arena's hipFree comes
        self.stream.synchronize()
        for graph, _ in self.graphs.values():
            graph.reset()
        if self.warm_graph is not None:
            self.warm_graph.reset()
        self.graphs = {}
        self.warm_graph = None
        self.weights = None
        self.x = self.y = self.h = self.workspace = None
        self.partials = self.seed_dev = self.warm_record = None
        self.arena = None
        self.torch.cuda.synchronize()
        self.torch.cuda.empty_cache()
        if self._stream_handle:
            self.mod.return_stream(self._stream_handle, self._device_index)
            self._stream_handle = 0
        self.stream = None
