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
pytest's own failure status).  Settings (``fail_under``, ``exclude_lines``,
``omit``) come from ``.coveragerc``, the file coverage.py reads too;
``--lcov`` writes an LCOV tracefile for Coveralls.
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


DEFAULT_EXCLUDE = ('pragma: no cover',)


def load_config(path=os.path.join(ROOT, '.coveragerc')):
    """``fail_under``, ``exclude_lines`` and ``omit`` from a coverage.py
    style ``.coveragerc`` (the same file serves coverage.py users)."""
    import configparser
    parser = configparser.ConfigParser()
    parser.read(path)

    def listed(section, key):
        raw = parser.get(section, key, fallback='')
        return [v.strip() for v in raw.splitlines() if v.strip()]
    return {
        'fail_under': parser.getfloat('report', 'fail_under', fallback=80.0),
        'exclude_lines': listed('report', 'exclude_lines') or list(
            DEFAULT_EXCLUDE),
        'omit': listed('run', 'omit') + listed('report', 'omit'),
    }


def _excluded(text, patterns):
    """Lines matching an ``exclude_lines`` regex; a matching block opener
    (``except ImportError:``) excludes the whole block, as coverage.py
    does."""
    import re
    regexes = [re.compile(p) for p in patterns]
    out = set()
    i = 0
    while i < len(text):
        line = text[i]
        if any(r.search(line) for r in regexes):
            out.add(i + 1)
            if line.rstrip().endswith(':'):
                indent = len(line) - len(line.lstrip())
                j = i + 1
                while j < len(text) and (not text[j].strip() or len(
                        text[j]) - len(text[j].lstrip()) > indent):
                    out.add(j + 1)
                    j += 1
                i = j
                continue
        i += 1
    return out


def executable_lines(path, exclude=DEFAULT_EXCLUDE):
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
    # a module docstring / first line counts as executed on import only
    return lines - _excluded(source.split('\n'), exclude)


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


def report(tracer, package=PACKAGE, exclude=DEFAULT_EXCLUDE, omit=()):
    import fnmatch
    rows = []
    total_exec = total_hit = 0
    for base, dirs, files in os.walk(package):
        dirs[:] = [d for d in dirs if d != '__pycache__']
        for name in sorted(files):
            if not name.endswith('.py'):
                continue
            path = os.path.join(base, name)
            rel = os.path.relpath(path, ROOT)
            if any(fnmatch.fnmatch(rel, pat) for pat in omit):
                continue
            lines = executable_lines(path, exclude)
            hit = tracer.hits.get(path, set()) & lines
            total_exec += len(lines)
            total_hit += len(hit)
            pct = 100.0 * len(hit) / len(lines) if lines else 100.0
            rows.append((os.path.relpath(path, ROOT), len(lines), len(hit),
                         pct))
    total = 100.0 * total_hit / total_exec if total_exec else 100.0
    return rows, total


def write_lcov(tracer, out_path, package=PACKAGE, exclude=DEFAULT_EXCLUDE,
               omit=()):
    """LCOV tracefile (Coveralls / genhtml input) of the same data."""
    import fnmatch
    records = []
    for path in sorted(_package_files(package)):
        rel = os.path.relpath(path, ROOT)
        if any(fnmatch.fnmatch(rel, pat) for pat in omit):
            continue
        lines = sorted(executable_lines(path, exclude))
        hits = tracer.hits.get(path, set())
        body = ['TN:', 'SF:%s' % rel]
        body += ['DA:%d,%d' % (n, 1 if n in hits else 0) for n in lines]
        body += ['LF:%d' % len(lines),
                 'LH:%d' % sum(1 for n in lines if n in hits),
                 'end_of_record']
        records.append('\n'.join(body))
    with open(out_path, 'w') as handle:
        handle.write('\n'.join(records) + '\n')


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    pytest_args = []
    if '--' in argv:
        split = argv.index('--')
        argv, pytest_args = argv[:split], argv[split + 1:]
    parser = argparse.ArgumentParser(description=__doc__.split('\n')[0])
    parser.add_argument('--fail-under', type=float, default=None,
                        help='default: .coveragerc [report] fail_under')
    parser.add_argument('--rcfile', default=os.path.join(ROOT, '.coveragerc'))
    parser.add_argument('--lcov', default=None,
                        help='also write an LCOV tracefile (Coveralls)')
    parser.add_argument('--output', default=None,
                        help='also write the table to this file')
    parser.add_argument('--missing', default='',
                        help='comma-separated file name fragments: list '
                             'their never-executed lines')
    args = parser.parse_args(argv)
    config = load_config(args.rcfile)
    if args.fail_under is None:
        args.fail_under = config['fail_under']
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
    rows, total = report(tracer, exclude=config['exclude_lines'],
                         omit=config['omit'])
    if args.lcov:
        write_lcov(tracer, args.lcov, exclude=config['exclude_lines'],
                   omit=config['omit'])
    lines = ['%-52s %6s %6s %6s' % ('file', 'stmts', 'hit', 'cover')]
    for path, n, hit, pct in rows:
        lines.append('%-52s %6d %6d %5.1f%%' % (path, n, hit, pct))
    lines.append('%-52s %6s %6s %5.1f%%' % ('TOTAL', '', '', total))
    for frag in filter(None, args.missing.split(',')):
        for path in sorted(p for p in _package_files() if frag in p):
            missed = sorted(executable_lines(path, config['exclude_lines'])
                            - tracer.hits.get(path, set()))
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
