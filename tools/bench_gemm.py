#!/usr/bin/env python3
"""GEMM microbenchmark: native gfx950 kernel vs torch.matmul (hipBLASLt).

Interleaves the two in one process (cdna_hip_programming.md rule 24) on
random data (rule 25) at the worker's shapes and prints one JSON line per
shape with TFLOP/s for each.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from kiosk_autoscaler_amd.ops import kernels, native
    mod = native.load()
    parser = argparse.ArgumentParser()
    parser.add_argument('--iters', type=int, default=20)
    parser.add_argument('--rounds', type=int, default=5)
    parser.add_argument('--shapes', default='2048x16384x4096,2048x4096x16384,'
                        '8192x16384x4096,4096x4096x4096')
    parser.add_argument('--only', default='',
                        help='comma-separated function names to time '
                             '(default: all)')
    parser.add_argument('--group-m', default='',
                        help='comma-separated tile-row group sizes of the '
                             '256-row kernels: each adds <name>_gm<G> arms '
                             'of the 4-wave kernels (A/B in one process)')
    parser.add_argument('--mfma32', action='store_true',
                        help='add <name>_m32 arms of the 4-wave kernels on '
                             'v_mfma_f32_32x32x16_bf16 (gemm_set_mfma32)')
    parser.add_argument('--pair', action='store_true',
                        help='add <name>_pair arms: the 4-wave path on the '
                             '8-wave, two-waves-per-SIMD kernel '
                             '(gemm_set_pair)')
    args = parser.parse_args()
    group_ms = [int(g) for g in args.group_m.split(',') if g]
    pair_modes = [1] if args.pair else []
    default_gm = mod.gemm_group_m()
    for spec in args.shapes.split(','):
        M, N, K = (int(v) for v in spec.split('x'))
        a = (torch.rand(M, K, device='cuda') * 2 - 1).to(torch.bfloat16)
        b = ((torch.rand(N, K, device='cuda') * 2 - 1) * 0.05).to(torch.bfloat16)
        bias = torch.randn(N, device='cuda')
        out = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)

        def ours():
            kernels.gemm(a, b, bias=bias, epilogue='gelu', out=out)

        def ours_plain():
            kernels.gemm(a, b, out=out, variant='128')

        def ours_256():
            kernels.gemm(a, b, out=out, variant='256')

        def ours_256w4():
            kernels.gemm(a, b, out=out, variant='256w4')

        def ours_256w4p():
            kernels.gemm(a, b, out=out, variant='256w4p')

        def ours_256w4p_gelu():
            kernels.gemm(a, b, bias=bias, epilogue='gelu', out=out,
                         variant='256w4p')

        def ours_256_gelu():
            kernels.gemm(a, b, bias=bias, epilogue='gelu', out=out,
                         variant='256')

        def ours_256w4_gelu():
            kernels.gemm(a, b, bias=bias, epilogue='gelu', out=out,
                         variant='256w4')

        def ours_256x128():
            kernels.gemm(a, b, out=out, variant='256x128')

        def ours_splitk():
            kernels.gemm(a, b, out=out, variant='256splitk')

        default_mode = mod.gemm_splitk_fused()

        def ours_splitk_fused():
            mod.gemm_set_splitk_fused(1)
            kernels.gemm(a, b, out=out, variant='256splitk')
            mod.gemm_set_splitk_fused(default_mode)

        def ours_splitk_reduce():
            mod.gemm_set_splitk_fused(0)
            kernels.gemm(a, b, out=out, variant='256splitk')
            mod.gemm_set_splitk_fused(default_mode)

        def theirs():
            torch.nn.functional.gelu(torch.addmm(bias.to(torch.bfloat16), a,
                                                 b.t()), approximate='tanh')

        def theirs_plain():
            torch.matmul(a, b.t(), out=out)

        bias_bf16 = bias.to(torch.bfloat16)

        def theirs_fused_gelu():
            # hipBLASLt with its own GELU_BIAS epilogue (tanh GELU)
            torch._addmm_activation(bias_bf16, a, b.t(), use_gelu=True)

        fns = {'native_gelu_auto': ours, 'native128': ours_plain,
               'torch_gelu': theirs, 'torch': theirs_plain,
               'hipblaslt_epilogue_gelu': theirs_fused_gelu}
        if N % 256 == 0:
            fns['native256'] = ours_256
            fns['native256w4'] = ours_256w4
            fns['native256_gelu'] = ours_256_gelu
            fns['native256w4_gelu'] = ours_256w4_gelu
            fns['native256w4p'] = ours_256w4p
            fns['native256w4p_gelu'] = ours_256w4p_gelu
        fns['native256x128'] = ours_256x128
        if mod.gemm_workspace_bytes(M, N, K):
            fns['native256splitk'] = ours_splitk
            fns['native256splitk_fused'] = ours_splitk_fused
            fns['native256splitk_reduce'] = ours_splitk_reduce

        for gm in group_ms:
            for base in ('native256w4', 'native256w4_gelu'):
                if base in fns:
                    def arm(fn=fns[base], gm=gm):
                        mod.gemm_set_group_m(gm)
                        fn()
                        mod.gemm_set_group_m(default_gm)
                    fns['%s_gm%d' % (base, gm)] = arm
        if args.mfma32:
            for base in ('native_gelu_auto', 'native256w4', 'native256w4_gelu',
                         'native256splitk'):
                if base in fns:
                    def arm32(fn=fns[base]):
                        mod.gemm_set_mfma32(1)
                        fn()
                        mod.gemm_set_mfma32(0)
                    fns[base + '_m32'] = arm32
        for mode in pair_modes:
            for base in ('native_gelu_auto', 'native256w4', 'native256w4_gelu',
                         'native256splitk'):
                if base in fns:
                    def arm_pair(fn=fns[base], mode=mode):
                        mod.gemm_set_pair(mode)
                        fn()
                        mod.gemm_set_pair(0)
                    fns['%s_pair' % base] = arm_pair
        if args.only:
            keep = set(args.only.split(','))
            fns = {k: v for k, v in fns.items() if k in keep}
        results = {k: [] for k in fns}
        for fn in fns.values():
            fn()
        torch.cuda.synchronize()
        for _ in range(args.rounds):
            for name, fn in fns.items():
                start = torch.cuda.Event(enable_timing=True)
                end = torch.cuda.Event(enable_timing=True)
                start.record()
                for _ in range(args.iters):
                    fn()
                end.record()
                end.synchronize()
                ms = start.elapsed_time(end) / args.iters
                results[name].append(2.0 * M * N * K / (ms * 1e-3) / 1e12)
        ref = (a.float() @ b.float().t())
        summary = {'shape': [M, N, K]}
        for name, fn in (('128', ours_plain), ('256', ours_256),
                         ('256w4', ours_256w4), ('256x128', ours_256x128)):
            if name in ('256', '256w4') and N % 256:
                continue
            out.zero_()
            fn()
            torch.cuda.synchronize()
            summary['max_abs_err_' + name] = (out.float() - ref).abs().max().item()
        for name, vals in results.items():
            vals.sort()
            summary[name + '_tflops_median'] = round(vals[len(vals) // 2], 1)
            summary[name + '_tflops_max'] = round(vals[-1], 1)
        print(json.dumps(summary), flush=True)


if __name__ == '__main__':
    main()
