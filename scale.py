"""Scale GPU worker processes on MI355X based on items in Redis queues.

Drop-in entry point with the reference's CLI contract (``python scale.py``,
configured only by environment variables; reference ``scale.py``).  See
:mod:`kiosk_autoscaler_amd.cli` for the loop and README.md for the
variables.
"""
from kiosk_autoscaler_amd.cli import main

if __name__ == '__main__':
    main()
