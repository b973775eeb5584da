#!/usr/bin/env python3
"""The worker's production forward for rocprofv3 --pmc, beside hipBLASLt.

Runs ``Engine.forward`` at the worker shape (auto GEMM dispatch: the 4-wave
256x256 bias+GELU up-projection, the split-K down-projection and its
reduce, inside the captured graph) ``--iters`` times, then the same GEMMs
through torch (hipBLASLt: ``addmm`` + GELU, ``addmm``) on random data of
the same shapes, so one profile holds both kernels' counters:

    rocprofv3 --pmc SQ_WAVE_CYCLES ... --kernel-trace --stats \\
        --output-format csv -d gpurun_out/pmc_fwd/a -- \\
        python3 tools/forward_pmc.py
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    parser = argparse.ArgumentParser()
    parser.add_argument('--rows', type=int, default=2048)
    parser.add_argument('--dim', type=int, default=4096)
    parser.add_argument('--hidden', type=int, default=16384)
    parser.add_argument('--layers', type=int, default=4)
    parser.add_argument('--iters', type=int, default=5)
    parser.add_argument('--no-torch', action='store_true')
    parser.add_argument('--calib-iters', type=int, default=200000,
                        help='warm-start kernel iterations (4 back-to-back '
                             'MFMAs each on every SIMD): the MFMA-busy '
                             'calibration kernel (0 = skip)')
    args = parser.parse_args()
    import torch
    from kiosk_autoscaler_amd.ops import native
    mod = native.load()
    if args.calib_iters:
        # calibration: every SIMD issues back-to-back MFMAs, so
        # SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x kernel cycles) should read ~1
        # (tools/pmc_summary.py); the records' s_memtime / s_memrealtime
        # give the shader clock under MFMA load
        w = torch.zeros(1 << 20, dtype=torch.bfloat16, device='cuda')
        rec = torch.zeros(256 * 8, dtype=torch.int32, device='cuda')
        mod.warmstart_raw(w.data_ptr(), w.numel(), rec.data_ptr(), 256,
                          args.calib_iters, 128 * 1024,
                          torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        r = rec.view(256, 8).cpu().numpy().astype('int64') & 0xffffffff
        real = ((r[:, 5] << 32) | r[:, 4]) - ((r[:, 3] << 32) | r[:, 2])
        ghz = (r[:, 7] / (real / 100e6)) / 1e9
        print('calib: %d MFMA/SIMD, shader clock %.3f GHz (min %.3f max '
              '%.3f), %.1f us' % (4 * args.calib_iters, ghz.mean(), ghz.min(),
                                  ghz.max(), real.mean() / 100.0), flush=True)
    engine = mod.Engine(0, args.dim, args.hidden, args.layers, args.rows, 3)
    try:
        engine.prepare(args.rows)
        for i in range(args.iters):
            out = engine.forward(args.rows, 1, i)
        print('engine forward %.3f ms' % out['gpu_ms'], flush=True)
    finally:
        engine.close()
    if args.no_torch:
        return
    g = torch.Generator(device='cuda').manual_seed(0)

    def rnd(*shape, scale=1.0):
        return ((torch.rand(*shape, generator=g, device='cuda') * 2 - 1) *
                scale).to(torch.bfloat16)
    x = rnd(args.rows, args.dim)
    w1 = rnd(args.hidden, args.dim, scale=args.dim ** -0.5)
    w2 = rnd(args.dim, args.hidden, scale=args.hidden ** -0.5)
    b1 = rnd(args.hidden)
    b2 = rnd(args.dim)
    for _ in range(args.iters):
        for _ in range(args.layers):
            h = torch.nn.functional.gelu(torch.addmm(b1, x, w1.t()),
                                         approximate='tanh')
            torch.addmm(b2, h, w2.t())
    torch.cuda.synchronize()
    print('torch (hipBLASLt) done', flush=True)


if __name__ == '__main__':
    main()
