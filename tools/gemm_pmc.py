#!/usr/bin/env python3
"""Launch one GEMM variant a fixed number of times, for rocprofv3 --pmc.

    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES \
        SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --stats \
        --output-format csv -d gpurun_out/pmc -- python3 tools/gemm_pmc.py
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    parser = argparse.ArgumentParser()
    parser.add_argument('--shapes', default='2048x16384x4096,2048x4096x16384')
    parser.add_argument('--variants', default='256,256x128,128')
    parser.add_argument('--iters', type=int, default=10)
    parser.add_argument('--mfma32', action='store_true',
                        help='run each 256w4 variant again on the 32x32x16 '
                             'kernel (gemm_set_mfma32; its own kernel name)')
    args = parser.parse_args()
    import torch
    from kiosk_autoscaler_amd.ops import kernels
    for spec in args.shapes.split(','):
        M, N, K = (int(v) for v in spec.split('x'))
        a = (torch.rand(M, K, device='cuda') * 2 - 1).to(torch.bfloat16)
        b = ((torch.rand(N, K, device='cuda') * 2 - 1) * 0.05).to(
            torch.bfloat16)
        out = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
        for variant in args.variants.split(','):
            if variant in ('256', '256w4') and N % 256:
                continue
            for _ in range(args.iters):
                kernels.gemm(a, b, out=out, variant=variant)
            torch.cuda.synchronize()
            print('%s %s done' % (spec, variant), flush=True)
            if args.mfma32 and variant == '256w4':
                from kiosk_autoscaler_amd.ops import native
                mod = native.load()
                mod.gemm_set_mfma32(1)
                for _ in range(args.iters):
                    kernels.gemm(a, b, out=out, variant=variant)
                torch.cuda.synchronize()
                mod.gemm_set_mfma32(0)
                print('%s %s mfma32 done' % (spec, variant), flush=True)


if __name__ == '__main__':
    main()
