#!/usr/bin/env python3
"""Where the PyTorch engine's first graph capture spends ~12 ms (its
``weights_on_device`` -> ``forward_captured`` stage in every woken standby's
prebuild; the second capture takes 0.14 ms).

Each case runs in a forked child of a parent that imported torch and the
native module without a HIP call (the zygote's shape); the child opens the
device like a standby (``preinit_device``), then times two captures of the
case's body on one stream.  Cases: ``kernel`` (one native memset),
``h2d`` / ``d2h`` (a pinned-memory copy node), ``forward`` (the engine's
whole forward), ``engine`` (the full ``TorchKioskEngine`` build, stages).
One JSON line per case.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def ms(t0):
    return round((time.perf_counter() - t0) * 1e3, 3)


def child(case, mod):
    import torch
    out = {'case': case}
    t0 = time.perf_counter()
    mod.preinit_device(0)
    out['preinit_ms'] = ms(t0)
    if case == 'native':
        t0 = time.perf_counter()
        engine = mod.Engine(0, 4096, 16384, 4, 2048, 1)
        out['build_ms'] = ms(t0)
        out['stages'] = dict(engine.stage_times())
        t0 = time.perf_counter()
        engine.forward(2048, 1, 0)
        out['first_forward_ms'] = ms(t0)
        engine.close()
        return out
    if case.startswith('dummy_'):
        # one throwaway graph of <kind> on its own stream first: does the
        # engine's first instantiate then drop to the second's cost?
        kind = case[len('dummy_'):]
        side = torch.cuda.Stream()
        scratch = torch.empty(4096, dtype=torch.uint8, device='cuda')
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        graph = mod.StreamGraph(side.cuda_stream)
        graph.begin()
        if kind == 'memset':
            mod.memset_async(scratch.data_ptr(), 0, 64, side.cuda_stream)
        elif kind == 'kernel':
            mod.init_uniform_f32(scratch.data_ptr(), 16, 1, -1.0, 1.0,
                                 side.cuda_stream)
        graph.end()
        out['dummy_ms'] = ms(t0)
        out['dummy_instantiate_ms'] = graph.instantiate_us / 1e3
        graph.reset()
        case = 'engine_calls'
    if case in ('engine', 'engine_calls', 'engine_warm_first'):
        from kiosk_autoscaler_amd.models.torch_kiosk import TorchKioskEngine
        from kiosk_autoscaler_amd.worker.runtime import WorkerConfig
        calls = []

        class Timed(object):
            """The native module, each call timed (first capture only)."""

            def __init__(self, real):
                self._real = real

            def __getattr__(self, name):
                fn = getattr(self._real, name)
                if not callable(fn):
                    return fn

                def timed(*args, **kw):
                    t = time.perf_counter()
                    try:
                        return fn(*args, **kw)
                    finally:
                        calls.append((name, ms(t)))
                return timed

        class Probe(TorchKioskEngine):
            def _enqueue_forward(self, rows):
                if case == 'engine' or calls:
                    return TorchKioskEngine._enqueue_forward(self, rows)
                real, self.mod = self.mod, Timed(self.mod)
                t = time.perf_counter()
                try:
                    return TorchKioskEngine._enqueue_forward(self, rows)
                finally:
                    self.mod = real
                    calls.append(('enqueue_total', ms(t)))

            def _record(self, enqueue):
                # TorchKioskEngine._record (native StreamGraph), timed
                t = time.perf_counter()
                graph = self.mod.StreamGraph(self.stream.cuda_stream)
                self.stream.synchronize()
                graph.begin()
                calls.append(('capture_begin', ms(t)))
                t = time.perf_counter()
                result = enqueue()
                calls.append(('enqueue', ms(t)))
                t = time.perf_counter()
                graph.end()
                calls.append(('capture_end', ms(t)))
                calls.append(('instantiate', graph.instantiate_us / 1e3))
                t = time.perf_counter()
                graph.launch()
                self.stream.synchronize()
                calls.append(('first_launch', ms(t)))
                return graph, result

        class WarmFirst(Probe):
            """The warm-start graph captured before the forward's."""

            def _capture(self, rows):
                if self.warm_graph is None:
                    self._capture_warm()
                return Probe._capture(self, rows)

            def _capture_warm(self):
                if self.warm_graph is None:
                    Probe._capture_warm(self)
        stages = {}
        t0 = time.perf_counter()
        cls = WarmFirst if case == 'engine_warm_first' else Probe
        engine = cls(WorkerConfig({}, {'worker_id': 'probe'}),
                     stage=lambda name: stages.setdefault(name, ms(t0)))
        out['stages'] = stages
        # a second forward graph (another row count): per-graph cost or
        # first-instantiate cost?
        t0 = time.perf_counter()
        engine._capture(1024)
        out['second_forward_graph_ms'] = ms(t0)
        if calls:
            out['calls'] = calls
        engine.close()
        return out
    handle = mod.take_stream(0)
    stream = torch.cuda.ExternalStream(handle) if handle else \
        torch.cuda.Stream()
    buf = torch.empty(1 << 20, dtype=torch.uint8, device='cuda')
    host = torch.zeros(1, dtype=torch.int64).pin_memory()
    dev = torch.zeros(1, dtype=torch.int64, device='cuda')
    torch.cuda.synchronize()

    def body():
        s = torch.cuda.current_stream().cuda_stream
        if case in ('kernel', 'h2d', 'd2h'):
            mod.memset_async(buf.data_ptr(), 0, 4096, s)
        if case == 'h2d':
            dev.copy_(host, non_blocking=True)
        if case == 'd2h':
            host.copy_(dev, non_blocking=True)

    for rep in ('first', 'second'):
        graph = torch.cuda.CUDAGraph()
        stream.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(stream):
            graph.capture_begin(capture_error_mode='thread_local')
            t1 = time.perf_counter()
            body()
            t2 = time.perf_counter()
            graph.capture_end()
        t3 = time.perf_counter()
        out[rep] = {'begin': round((t1 - t0) * 1e3, 3),
                    'body': round((t2 - t1) * 1e3, 3),
                    'end': round((t3 - t2) * 1e3, 3)}
        t0 = time.perf_counter()
        graph.replay()
        stream.synchronize()
        out[rep]['replay'] = ms(t0)
    return out


def main():
    cases = sys.argv[1].split(',') if len(sys.argv) > 1 else \
        ['kernel', 'h2d', 'd2h', 'engine', 'engine_calls']
    import torch  # noqa: F401  (before the native module: one HIP runtime)
    from kiosk_autoscaler_amd.ops import native
    mod = native.load(torch_first=True)
    for case in cases:
        r, w = os.pipe()
        pid = os.fork()
        if pid == 0:
            os.close(r)
            try:
                row = child(case, mod)
            except Exception as err:  # pylint: disable=broad-except
                row = {'case': case, 'error': repr(err)}
            os.write(w, (json.dumps(row) + '\n').encode())
            os._exit(0)
        os.close(w)
        data = b''
        while True:
            chunk = os.read(r, 65536)
            if not chunk:
                break
            data += chunk
        os.close(r)
        os.waitpid(pid, 0)
        print(data.decode().strip(), flush=True)
    return 0


if __name__ == '__main__':
    sys.exit(main())
