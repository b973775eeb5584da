#!/usr/bin/env python3
"""Line-coverage gate for ``kiosk_autoscaler_amd`` (the reference enforces
``--cov autoscaler`` with ``fail_under = 80``: ``/root/reference/
.coveragerc:12,15``, ``.github/workflows/tests.yaml:44``).

``coverage``/``pytest-cov`` are not installable in this image, so this is a
dependency-free tracer: ``sys.settrace`` + ``threading.settrace`` record the
lines executed in the package while pytest runs *in this process*;
executable lines come from the compiled code objects (``co_lines``), minus
lines marked ``# pragma: no cover``.  Child processes (mock workers spawned
by the integration tests, the CLI) are traced too: ``tools/covtrace_site``
goes on ``PYTHONPATH`` and its ``sitecustomize`` dumps each child's lines
(the pytest-cov subprocess hook, without the dependency).

    python tools/covtrace.py --fail-under 80 -- tests -m "not gpu" -q

prints a per-file table and the total and exits 1 below the gate (or with
pytest's own failure status).
"""
import argparse
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PACKAGE = os.path.join(ROOT, 'kiosk_autoscaler_amd')


class LineTracer(object):
    def __init__(self, prefix):
        self.prefix = prefix
        self.hits = {}

    def _global(self, frame, event, arg):
        filename = frame.f_code.co_filename
        if not filename.startswith(self.prefix):
            return None
        lines = self.hits.setdefault(filename, set())
        lines.add(frame.f_lineno)

        def local(frame, event, arg):
            if event == 'line':
                lines.add(frame.f_lineno)
            return local
        return local

    def start(self):
        # nested tracers (tests of this tool) restore the outer one on stop
        gettrace = getattr(threading, 'gettrace', lambda: None)
        self._saved = (sys.gettrace(), gettrace())
        threading.settrace(self._global)
        sys.settrace(self._global)

    def stop(self):
        outer, outer_threads = getattr(self, '_saved', (None, None))
        sys.settrace(outer)
        threading.settrace(outer_threads)


def _dump(tracer, directory):
    import json
    path = os.path.join(directory, 'cov-%d-%d.json' % (
        os.getpid(), threading.get_ident()))
    with open(path, 'w') as handle:
        json.dump({k: sorted(v) for k, v in tracer.hits.items()}, handle)


def start_child(directory):
    """Trace this (child) process; dump at exit, including ``os._exit``."""
    import atexit
    tracer = LineTracer(PACKAGE)
    tracer.start()
    done = []

    def dump():
        if not done:
            done.append(True)
            tracer.stop()
            try:
                _dump(tracer, directory)
            except OSError:
                pass
    atexit.register(dump)
    real_exit = os._exit

    def _exit(code):
        dump()
        real_exit(code)
    os._exit = _exit


def merge_children(tracer, directory):
    import json
    for name in os.listdir(directory):
        if not name.endswith('.json'):
            continue
        try:
            with open(os.path.join(directory, name)) as handle:
                data = json.load(handle)
        except (OSError, ValueError):
            continue
        for path, lines in data.items():
            tracer.hits.setdefault(path, set()).update(lines)


def executable_lines(path):
    with open(path, encoding='utf-8') as handle:
        source = handle.read()
    code = compile(source, path, 'exec')
    lines = set()
    stack = [code]
    while stack:
        co = stack.pop()
        for _, _, line in co.co_lines():
            if line is not None:
                lines.add(line)
        stack.extend(c for c in co.co_consts if hasattr(c, 'co_lines'))
    text = source.split('\n')
    excluded = {i + 1 for i, line in enumerate(text)
                if 'pragma: no cover' in line}
    # a module docstring / first line counts as executed on import only
    return lines - excluded


def _package_files(package=PACKAGE):
    for base, dirs, files in os.walk(package):
        dirs[:] = [d for d in dirs if d != '__pycache__']
        for name in files:
            if name.endswith('.py'):
                yield os.path.join(base, name)


def _ranges(numbers):
    out, start, prev = [], None, None
    for n in numbers:
        if start is None:
            start = prev = n
        elif n == prev + 1:
            prev = n
        else:
            out.append(str(start) if start == prev else '%d-%d' % (start,
                                                                    prev))
            start = prev = n
    if start is not None:
        out.append(str(start) if start == prev else '%d-%d' % (start, prev))
    return ','.join(out)


def report(tracer, package=PACKAGE):
    rows = []
    total_exec = total_hit = 0
    for base, dirs, files in os.walk(package):
        dirs[:] = [d for d in dirs if d != '__pycache__']
        for name in sorted(files):
            if not name.endswith('.py'):
                continue
            path = os.path.join(base, name)
            lines = executable_lines(path)
            hit = tracer.hits.get(path, set()) & lines
            total_exec += len(lines)
            total_hit += len(hit)
            pct = 100.0 * len(hit) / len(lines) if lines else 100.0
            rows.append((os.path.relpath(path, ROOT), len(lines), len(hit),
                         pct))
    total = 100.0 * total_hit / total_exec if total_exec else 100.0
    return rows, total


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    pytest_args = []
    if '--' in argv:
        split = argv.index('--')
        argv, pytest_args = argv[:split], argv[split + 1:]
    parser = argparse.ArgumentParser(description=__doc__.split('\n')[0])
    parser.add_argument('--fail-under', type=float, default=80.0)
    parser.add_argument('--output', default=None,
                        help='also write the table to this file')
    parser.add_argument('--missing', default='',
                        help='comma-separated file name fragments: list '
                             'their never-executed lines')
    args = parser.parse_args(argv)
    sys.path.insert(0, ROOT)
    import tempfile
    import pytest
    child_dir = tempfile.mkdtemp(prefix='kiosk-cov-')
    os.environ['KIOSK_COVTRACE_DIR'] = child_dir
    site = os.path.join(ROOT, 'tools', 'covtrace_site')
    os.environ['PYTHONPATH'] = os.pathsep.join(
        [site] + [p for p in os.environ.get('PYTHONPATH', '').split(
            os.pathsep) if p])
    tracer = LineTracer(PACKAGE)
    tracer.start()
    try:
        status = pytest.main(pytest_args or ['tests', '-m', 'not gpu', '-q'])
    finally:
        tracer.stop()
    merge_children(tracer, child_dir)
    rows, total = report(tracer)
    lines = ['%-52s %6s %6s %6s' % ('file', 'stmts', 'hit', 'cover')]
    for path, n, hit, pct in rows:
        lines.append('%-52s %6d %6d %5.1f%%' % (path, n, hit, pct))
    lines.append('%-52s %6s %6s %5.1f%%' % ('TOTAL', '', '', total))
    for frag in filter(None, args.missing.split(',')):
        for path in sorted(p for p in _package_files() if frag in p):
            missed = sorted(executable_lines(path) -
                            tracer.hits.get(path, set()))
            lines.append('missing %s: %s' % (os.path.relpath(path, ROOT),
                                             _ranges(missed)))
    text = '\n'.join(lines)
    print(text)
    if args.output:
        with open(args.output, 'w') as handle:
            handle.write(text + '\n')
    if status != 0:
        return int(status)
    if total < args.fail_under:
        print('FAIL: coverage %.1f%% is below fail_under=%.0f%%'
              % (total, args.fail_under))
        return 1
    return 0


if __name__ == '__main__':
    sys.exit(main())
