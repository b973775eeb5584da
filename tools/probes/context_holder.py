#!/usr/bin/env python3
"""Hold a bare HIP context (plus code objects) on GPU 0 for N seconds: the
second arm of the cold device-open probe (tools/preinit_probe.py) -- a GPU
that another process already has open.

    python3 tools/context_holder.py 60 &
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))


def main():
    from kiosk_autoscaler_amd.ops import native
    native.load().preload_modules(0)
    print('holding', flush=True)
    time.sleep(float(sys.argv[1]) if len(sys.argv) > 1 else 60.0)


if __name__ == '__main__':
    main()
