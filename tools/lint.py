"""Self-contained lint (the image has no flake8 / pycodestyle / clang-format;
``tools/lint.sh`` uses them when they are installed, with the settings in
``setup.cfg`` / ``.clang-format``).

Python (pycodestyle / pyflakes subset, as the reference CI's
``pycodestyle --ignore=E731`` + ``flake8``, ``.travis.yml:31-32``):
  E501 line > 79, W291/W293 trailing whitespace, W191 tab indentation,
  E303 more than two blank lines,
  W391/W292 file must end with exactly one newline, E999 syntax error,
  F401 imported name never used (``# noqa`` and ``__init__.py`` re-exports
  excepted), F811 duplicate top-level def.
C++ / HIP (``csrc/``): line > 100,
  (``.clang-format`` ColumnLimit), tabs, trailing whitespace, and the
  MI355X-only rules - no CUDA headers, no ``__CUDA_ARCH__`` and no
  ``__HIP_PLATFORM_*`` dual-path conditionals.

    python tools/lint.py [paths...]      # exit 1 on findings
"""
import ast
import os
import os.path as osp
import re
import sys

ROOT = osp.dirname(osp.dirname(osp.abspath(__file__)))
DEFAULT = ['deep_graph_matching_consensus_amd', 'tests', 'tools', 'examples',
           'bench.py', '__graft_entry__.py', 'setup.py', 'csrc']
SKIP_DIRS = {'build', '__pycache__', '.git', 'gpurun_out', '.ab_base'}
PY_MAX, CC_MAX = 79, 100
CC_EXT = ('.hip', '.cpp', '.h', '.hpp', '.cc')
CC_FORBIDDEN = [
    (re.compile(r'#\s*include\s*[<"]cuda'), 'CUDA header'),
    (re.compile(r'__CUDA_ARCH__'), '__CUDA_ARCH__ dual path'),
    (re.compile(r'#\s*if.*__HIP_PLATFORM_'), '__HIP_PLATFORM_ dual path'),
]


def _files(paths):
    for p in paths:
        p = osp.join(ROOT, p) if not osp.isabs(p) else p
        if osp.isfile(p):
            yield p
            continue
        for d, dirs, files in os.walk(p):
            dirs[:] = [x for x in dirs if x not in SKIP_DIRS]
            for f in sorted(files):
                if f.endswith('.py') or f.endswith(CC_EXT):
                    yield osp.join(d, f)


def _common(path, text, limit):
    out = []
    lines = text.split('\n')
    blank = 0
    for i, line in enumerate(lines, 1):
        blank = blank + 1 if not line.strip() else 0
        if blank == 3 and i < len(lines):
            out.append((i, 'E303 too many blank lines (3)'))
        if len(line) > limit:
            out.append((i, 'E501 line too long ({} > {})'.format(len(line),
                                                               limit)))
        if line.rstrip() != line:
            out.append((i, 'W291 trailing whitespace'))
        if '\t' in line[:len(line) - len(line.lstrip())]:
            out.append((i, 'W191 tab indentation'))
    if text and not text.endswith('\n'):
        out.append((len(lines), 'W292 no newline at end of file'))
    elif text.endswith('\n\n'):
        out.append((len(lines), 'W391 blank line at end of file'))
    return out


class _Names(ast.NodeVisitor):
    def __init__(self):
        self.used = set()

    def visit_Name(self, node):
        self.used.add(node.id)

    def visit_Attribute(self, node):
        base = node
        while isinstance(base, ast.Attribute):
            base = base.value
        if isinstance(base, ast.Name):
            self.used.add(base.id)
        self.generic_visit(node)


def _python(path, text):
    out = _common(path, text, PY_MAX)
    try:
        tree = ast.parse(text, filename=path)
    except SyntaxError as e:
        return out + [(e.lineno or 0, 'E999 syntax error: {}'.format(e.msg))]
    lines = text.split('\n')
    names = _Names()
    names.visit(tree)
    # Names listed in __all__ or used in string annotations count as used.
    for node in ast.walk(tree):
        if isinstance(node, ast.Constant) and isinstance(node.value, str):
            names.used.update(re.findall(r'[A-Za-z_]\w*', node.value))
    init = osp.basename(path) == '__init__.py'
    for node in tree.body:
        if not isinstance(node, (ast.Import, ast.ImportFrom)) or init:
            continue
        if 'noqa' in lines[node.lineno - 1] or (
                node.end_lineno and 'noqa' in lines[node.end_lineno - 1]):
            continue
        for alias in node.names:
            name = (alias.asname or alias.name).split('.')[0]
            if name == '*' or name.startswith('_'):
                continue
            if name not in names.used:
                out.append((node.lineno,
                            'F401 {!r} imported but unused'.format(name)))
    seen = {}
    for node in tree.body:
        if isinstance(node, (ast.FunctionDef, ast.ClassDef)):
            if node.name in seen:
                out.append((node.lineno, 'F811 redefinition of {!r} from '
                            'line {}'.format(node.name, seen[node.name])))
            seen[node.name] = node.lineno
    return out


def _cc(path, text):
    out = _common(path, text, CC_MAX)
    for i, line in enumerate(text.split('\n'), 1):
        for pat, what in CC_FORBIDDEN:
            if pat.search(line):
                out.append((i, 'X001 ' + what + ' (MI355X-only code)'))
    return out


def lint(paths=None):
    findings = []
    for f in _files(paths or DEFAULT):
        with open(f, encoding='utf-8') as fh:
            text = fh.read()
        res = _python(f, text) if f.endswith('.py') else _cc(f, text)
        findings += [(osp.relpath(f, ROOT), ln, msg) for ln, msg in res]
    return findings


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    findings = lint(argv or None)
    for f, ln, msg in findings:
        print('{}:{}: {}'.format(f, ln, msg))
    print('{} finding(s)'.format(len(findings)))
    return 1 if findings else 0


if __name__ == '__main__':
    sys.exit(main())
