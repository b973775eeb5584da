"""Quality gates of the reference, restored (``pytest --pep8`` at 85
columns: ``/root/reference/pytest.ini:22-25``; coverage ``fail_under = 80``:
``.coveragerc:12``).  The lint runs here on every test run; the coverage
gate is ``tools/covtrace.py`` (CI), checked here for its mechanics."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tools'))

import covtrace  # noqa: E402
import lint  # noqa: E402


def test_repository_is_lint_clean():
    report = lint.run()
    assert report == [], '\n'.join(report)


def test_lint_catches_each_rule(tmp_path):
    bad = tmp_path / 'bad.py'
    bad.write_text('import os\nimport sys  # noqa\n'
                   'x = 1 \n'
                   'if x == None:\n    pass\n'
                   'try:\n    pass\nexcept:\n    pass\n'
                   'y = "%s"\n' % ('a' * 90))
    codes = [code for _, code, _ in lint.check_file(str(bad))]
    assert sorted(codes) == ['E501', 'E711', 'E722', 'F401', 'W291']
    broken = tmp_path / 'broken.py'
    broken.write_text('def f(:\n')
    assert [c for _, c, _ in lint.check_file(str(broken))] == ['E999']


def test_covtrace_counts_lines(tmp_path):
    pkg = tmp_path / 'pkg'
    pkg.mkdir()
    mod = pkg / 'm.py'
    mod.write_text('def f(a):\n    if a:\n        return 1\n'
                   '    return 2  # pragma: no cover\n')
    tracer = covtrace.LineTracer(str(pkg))
    sys.path.insert(0, str(tmp_path))
    outer = sys.gettrace()      # covtrace's own tracer when run under it
    try:
        tracer.start()
        import pkg.m as m  # noqa: F401
        m.f(True)
        tracer.stop()
    finally:
        sys.path.remove(str(tmp_path))
    # a nested tracer hands the process back to the outer one: stopping it
    # used to switch the gate's tracing off for the rest of the session
    assert sys.gettrace() is outer
    rows, total = covtrace.report(tracer, str(pkg))
    assert rows and total == 100.0   # line 4 excluded by the pragma


def test_native_module_imports_without_a_gpu():
    """The gfx950 extension loads on a CPU host (kernels are not run)."""
    from kiosk_autoscaler_amd.ops import native
    so = [f for f in os.listdir(os.path.join(ROOT, 'kiosk_autoscaler_amd',
                                             'ops')) if f.endswith('.so')]
    if not so:
        import pytest
        pytest.skip('extension not built')
    mod = native.load()
    assert mod.arch == 'gfx950'
    assert callable(mod.mem_info) and hasattr(mod, 'Fence')


def test_lint_cli_exit_status():
    proc = subprocess.run([sys.executable, os.path.join(ROOT, 'tools',
                                                        'lint.py')],
                          stdout=subprocess.PIPE, text=True, timeout=120)
    assert proc.returncode == 0, proc.stdout


def test_covtrace_config_exclusions_and_lcov(tmp_path):
    """``.coveragerc`` drives the gate (fail_under, exclude_lines with
    coverage.py's block semantics, omit) and ``--lcov`` output is a valid
    tracefile."""
    rc = tmp_path / 'rc'
    rc.write_text('[run]\nomit =\n    pkg/skip.py\n[report]\nfail_under = 91\n'
                  'exclude_lines =\n    pragma: no cover\n'
                  '    except ImportError\n')
    config = covtrace.load_config(str(rc))
    assert config['fail_under'] == 91.0
    assert config['omit'] == ['pkg/skip.py']
    text = ['try:', '    import x', 'except ImportError:', '    x = None',
            '    y = 1', 'z = 2  # pragma: no cover', 'w = 3']
    assert covtrace._excluded(text, config['exclude_lines']) == {3, 4, 5, 6}
    # the repository's own file parses and keeps the reference's gate
    assert covtrace.load_config()['fail_under'] == 80.0

    tracer = covtrace.LineTracer('/nonexistent')
    pkg = os.path.join(ROOT, 'kiosk_autoscaler_amd')
    policy = os.path.join(pkg, 'policy.py')
    tracer.hits[policy] = {1, 2, 3}
    out = tmp_path / 'lcov.info'
    covtrace.write_lcov(tracer, str(out), package=pkg,
                        omit=['kiosk_autoscaler_amd/[!p]*',
                              'kiosk_autoscaler_amd/p[!o]*'])
    records = out.read_text().strip().split('end_of_record')
    assert records[0].startswith('TN:\nSF:kiosk_autoscaler_amd/policy.py')
    assert 'LF:' in records[0] and 'LH:' in records[0]
