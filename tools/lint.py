#!/usr/bin/env python3
"""Style/lint gate (the reference runs ``pytest --pep8`` with a max line
length of 85, ``/root/reference/pytest.ini:22-25``, ``tests.yaml:44``).

No flake8/pycodestyle/pylint is installable here, so this is a small,
dependency-free checker of the rules that matter for this code base:

* E501 line longer than ``--max-line-length`` (85, the reference's value)
* W191 tab indentation, W291 trailing whitespace, W292/W391 end of file
* E711/E712 ``==``/``!=`` against ``None``/``True``/``False``
* E722 bare ``except:``
* E999 the file does not compile
* F401 a module-level import never used (``__init__.py`` re-exports,
  ``__all__`` members and ``# noqa`` lines are exempt)

``python tools/lint.py [paths...]`` prints ``path:line: CODE message`` and
exits 1 when anything is found; ``tests/test_lint.py`` runs it on the repo.
"""
import argparse
import ast
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_PATHS = ('kiosk_autoscaler_amd', 'tests', 'tools', 'bench.py',
                 'scale.py', '__graft_entry__.py')


def iter_files(paths):
    for path in paths:
        full = os.path.join(ROOT, path) if not os.path.isabs(path) else path
        if os.path.isfile(full):
            yield full
            continue
        for base, dirs, files in os.walk(full):
            dirs[:] = [d for d in dirs if d not in ('__pycache__', 'build')]
            for name in sorted(files):
                if name.endswith('.py'):
                    yield os.path.join(base, name)


def _noqa(line):
    return '# noqa' in line


def _unused_imports(tree, lines, is_init):
    if is_init:
        return []
    imported = {}
    for node in tree.body:
        if isinstance(node, (ast.Import, ast.ImportFrom)):
            if isinstance(node, ast.ImportFrom) and node.module == '__future__':
                continue
            for alias in node.names:
                if alias.name == '*':
                    continue
                name = alias.asname or alias.name.split('.')[0]
                imported[name] = node.lineno
    if not imported:
        return []
    used = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Name):
            used.add(node.id)
        elif isinstance(node, ast.Attribute):
            root = node
            while isinstance(root, ast.Attribute):
                root = root.value
            if isinstance(root, ast.Name):
                used.add(root.id)
    exported = set()
    for node in tree.body:
        if isinstance(node, ast.Assign) and any(
                isinstance(t, ast.Name) and t.id == '__all__'
                for t in node.targets):
            try:
                exported.update(ast.literal_eval(node.value))
            except ValueError:
                pass
    out = []
    for name, lineno in sorted(imported.items(), key=lambda kv: kv[1]):
        if name in used or name in exported or _noqa(lines[lineno - 1]):
            continue
        out.append((lineno, 'F401', "'%s' imported but unused" % name))
    return out


def _ast_checks(tree, lines):
    out = []
    for node in ast.walk(tree):
        if isinstance(node, ast.ExceptHandler) and node.type is None:
            if not _noqa(lines[node.lineno - 1]):
                out.append((node.lineno, 'E722', 'bare except'))
        elif isinstance(node, ast.Compare):
            for op, right in zip(node.ops, node.comparators):
                if not isinstance(op, (ast.Eq, ast.NotEq)) or \
                        not isinstance(right, ast.Constant):
                    continue
                value = right.value
                if value is None:
                    code = 'E711'
                elif isinstance(value, bool):
                    code = 'E712'
                else:
                    continue
                if not _noqa(lines[node.lineno - 1]):
                    out.append((node.lineno, code,
                                'comparison to %r with ==/!=' % value))
    return out


def check_file(path, max_line=85):
    with open(path, encoding='utf-8') as handle:
        text = handle.read()
    lines = text.split('\n')
    findings = []
    for i, line in enumerate(lines, 1):
        if len(line) > max_line and not _noqa(line):
            findings.append((i, 'E501', 'line too long (%d > %d)' % (
                len(line), max_line)))
        if line.rstrip() != line:
            findings.append((i, 'W291', 'trailing whitespace'))
        if line[:len(line) - len(line.lstrip())].count('\t'):
            findings.append((i, 'W191', 'indentation contains tabs'))
    if text and not text.endswith('\n'):
        findings.append((len(lines), 'W292', 'no newline at end of file'))
    elif text.endswith('\n\n'):
        findings.append((len(lines) - 1, 'W391', 'blank line at end of file'))
    try:
        tree = ast.parse(text, filename=path)
    except SyntaxError as err:
        findings.append((err.lineno or 1, 'E999', 'SyntaxError: %s' % err.msg))
        return findings
    findings += _ast_checks(tree, lines)
    findings += _unused_imports(tree, lines,
                                os.path.basename(path) == '__init__.py')
    return sorted(findings)


def run(paths=DEFAULT_PATHS, max_line=85):
    report = []
    for path in iter_files(paths):
        for lineno, code, message in check_file(path, max_line):
            report.append('%s:%d: %s %s' % (os.path.relpath(path, ROOT),
                                            lineno, code, message))
    return report


def main(argv=None):
    parser = argparse.ArgumentParser(description=__doc__.split('\n')[0])
    parser.add_argument('paths', nargs='*', default=list(DEFAULT_PATHS))
    parser.add_argument('--max-line-length', type=int, default=85)
    args = parser.parse_args(argv)
    report = run(args.paths, args.max_line_length)
    for line in report:
        print(line)
    return 1 if report else 0


if __name__ == '__main__':
    sys.exit(main())
