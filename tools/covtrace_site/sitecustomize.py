"""Child-process hook of tools/covtrace.py (the pytest-cov subprocess
analog): when ``KIOSK_COVTRACE_DIR`` is set, every Python process started
with this directory on ``PYTHONPATH`` -- the mock workers the integration
tests spawn, the autoscaler CLI -- traces the package's lines and dumps them
there on exit (``atexit`` and ``os._exit``, which the workers use)."""
import os

if os.environ.get('KIOSK_COVTRACE_DIR'):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))))
    import covtrace
    covtrace.start_child(os.environ['KIOSK_COVTRACE_DIR'])
