"""Example plug-in engine: the worker MLP as a plain PyTorch model.

``WORKER_ENGINE=kiosk_autoscaler_amd.models.torch_engine:TorchMlpEngine``
serves the same architecture as the built-in engine (``MODEL_DIM`` ->
``MODEL_HIDDEN`` -> ``MODEL_DIM``, tanh-GELU, residual, ``MODEL_LAYERS``
blocks, bf16, random init) through ``torch.nn`` on the worker's pinned GPU
-- the shape of a user bringing their own PyTorch model to the framework
(see :mod:`.plugin`).  Each job's ``rows`` x ``MODEL_DIM`` input is drawn
from its ``seed``; the result written back is the output's fp32 sum and
mean absolute value.  The built-in engine (hand-written gfx950 GEMMs,
captured hipGraph) remains the default and the faster one.
"""
import math


class TorchMlpEngine(object):

    def __init__(self, cfg, stage=None):
        import torch
        self.torch = torch
        self.device = torch.device('cuda' if torch.cuda.is_available()
                                   else 'cpu')
        self.dtype = torch.bfloat16
        self.dim, self.hidden = cfg.dim, cfg.hidden
        self.max_rows = max(cfg.rows * cfg.batch, 1)
        # weights are created and randomised on the device: a GB of
        # parameters initialised on the host would dominate the first
        # scale-up (the built-in engine does the same with its init kernel)
        gen = torch.Generator(device=self.device).manual_seed(cfg.seed)
        factory = {'device': self.device, 'dtype': self.dtype}
        layers = []
        for _ in range(cfg.layers):
            up = torch.nn.Linear(cfg.dim, cfg.hidden, **factory)
            down = torch.nn.Linear(cfg.hidden, cfg.dim, **factory)
            for lin in (up, down):
                bound = 1.0 / math.sqrt(lin.in_features)
                with torch.no_grad():
                    lin.weight.uniform_(-bound, bound, generator=gen)
                    lin.bias.uniform_(-bound, bound, generator=gen)
            layers.append(torch.nn.ModuleList([up, down]))
        self.layers = torch.nn.ModuleList(layers)
        self.layers.eval()
        if stage:
            stage('weights_on_device')

    def _forward(self, x):
        gelu = self.torch.nn.functional.gelu
        for up, down in self.layers:
            x = down(gelu(up(x), approximate='tanh')) + x
        return x

    def _input(self, rows, seed):
        torch = self.torch
        gen = torch.Generator(device='cpu').manual_seed(int(seed))
        x = torch.rand(rows, self.dim, generator=gen) * 2 - 1
        return x.to(self.device, self.dtype)

    def warmstart(self):
        with self.torch.inference_mode():
            self._forward(self._input(8, 0))
        if self.device.type == 'cuda':
            self.torch.cuda.synchronize()
        return {'backend': 'torch', 'device': str(self.device)}

    def infer(self, jobs):
        """One forward per job; a job with ``service_ms`` (the benchmark's
        fixed per-key GPU time) repeats the forward until that much time
        has passed, like the built-in engine's ``forward_for``."""
        import time
        torch = self.torch
        out = []
        with torch.inference_mode():
            for job in jobs:
                t0 = time.perf_counter()
                x = self._input(job['rows'], job['seed'])
                y = self._forward(x)
                passes = 1
                budget = float(job.get('service_ms') or 0) / 1e3
                while budget > 0:
                    if self.device.type == 'cuda':
                        torch.cuda.synchronize()
                    if time.perf_counter() - t0 >= budget:
                        break
                    y = self._forward(x)
                    passes += 1
                yf = y.float()
                out.append({'output_sum': '%.6e' % float(yf.sum()),
                            'output_mean_abs': '%.6e' % float(
                                yf.abs().mean()),
                            'passes': passes, 'engine': 'torch'})
        return out

    def reference(self, rows, seed):
        """The same forward in fp32 (tests)."""
        torch = self.torch
        x = self._input(rows, seed).float()
        with torch.inference_mode():
            for up, down in self.layers:
                h = torch.nn.functional.linear(x, up.weight.float(),
                                               up.bias.float())
                h = torch.nn.functional.gelu(h, approximate='tanh')
                x = torch.nn.functional.linear(h, down.weight.float(),
                                               down.bias.float()) + x
        return x

    def close(self):
        self.layers = None
        if self.device.type == 'cuda':
            self.torch.cuda.empty_cache()
