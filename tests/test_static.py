"""Static gates (the reference's flake8 / isort / strict-mypy CI, ``setup.cfg:26-68``).

flake8 and mypy are not installed in this image, so the same classes of defects are
checked with the standard library:

* every Python file compiles and no line is longer than 99 columns (flake8's limit in
  the reference; a trailing ``# type: ignore[...]`` pragma does not count);
* no unused imports (pyflakes F401; ``__init__`` re-exports and ``# noqa`` excepted);
* every public function and method of the package annotates all parameters and its
  return type (the part of ``mypy --strict``'s ``disallow_untyped_defs`` /
  ``disallow_incomplete_defs`` that needs no type inference);
* no ``print`` in library code outside ``__main__`` blocks and the build script;
* the module-level imports of the package follow the reference's isort setting
  (``force_sort_within_sections``): ``__future__``, standard library, third party, this
  package, each section sorted by module name regardless of ``import`` / ``from``.
"""
import ast
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PACKAGE = os.path.join(ROOT, 'torchgpipe_amd')
PRAGMA = re.compile(r'\s*#\s*(type:\s*ignore(\[[^\]]*\])?|noqa(:\s*[A-Z0-9, ]+)?)\s*$')


def _python_files(*dirs: str):
    out = []
    for d in dirs:
        for dirpath, _, files in os.walk(os.path.join(ROOT, d)):
            if '__pycache__' in dirpath:
                continue
            out += [os.path.join(dirpath, f) for f in files if f.endswith('.py')]
    return sorted(out)


ALL = _python_files('torchgpipe_amd', 'tests', 'benchmarks', 'scripts') + [
    os.path.join(ROOT, f) for f in ('bench.py', '__graft_entry__.py',
                                    'torchgpipe_amd_balancing.py')]
LIB = _python_files('torchgpipe_amd')


def _rel(path: str) -> str:
    return os.path.relpath(path, ROOT)


@pytest.mark.parametrize('path', ALL, ids=_rel)
def test_compiles_and_line_length(path):
    src = open(path).read()
    compile(src, path, 'exec')
    long = [i for i, line in enumerate(src.splitlines(), 1)
            if len(PRAGMA.sub('', line)) > 99]
    assert not long, f'{_rel(path)}: lines longer than 99 columns: {long}'


def _unused_imports(path: str):
    src = open(path).read()
    tree = ast.parse(src)
    lines = src.splitlines()
    imported = {}
    for node in ast.walk(tree):
        if isinstance(node, (ast.Import, ast.ImportFrom)):
            if 'noqa' in lines[node.lineno - 1]:
                continue
            for alias in node.names:
                name = (alias.asname or alias.name).split('.')[0]
                if name != '*':
                    imported[name] = node.lineno
    used = set()
    strings = []
    for node in ast.walk(tree):
        if isinstance(node, ast.Name):
            used.add(node.id)
        elif isinstance(node, ast.Attribute):
            root = node
            while isinstance(root, ast.Attribute):
                root = root.value
            if isinstance(root, ast.Name):
                used.add(root.id)
        elif isinstance(node, ast.Constant) and isinstance(node.value, str):
            strings.append(node.value)  # __all__ entries, string annotations
    return [(name, line) for name, line in imported.items()
            if name not in used and not any(name in s for s in strings)]


@pytest.mark.parametrize('path', [p for p in ALL if not p.endswith('__init__.py')], ids=_rel)
def test_no_unused_imports(path):
    assert not _unused_imports(path), f'{_rel(path)}: {_unused_imports(path)}'


@pytest.mark.parametrize('path', LIB, ids=_rel)
def test_public_functions_are_annotated(path):
    src = open(path).read()
    lines = src.splitlines()
    missing = []
    for node in ast.walk(ast.parse(src)):
        if not isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef)):
            continue
        if node.name.startswith('_') and not node.name.startswith('__'):
            continue
        if 'type: ignore' in lines[node.lineno - 1]:
            continue  # explicitly waived (autograd ctx signatures, etc.)
        args = node.args.args + node.args.kwonlyargs
        bare = [a.arg for a in args
                if a.annotation is None and a.arg not in ('self', 'cls', 'ctx')]
        if bare or node.returns is None:
            missing.append((node.lineno, node.name, bare))
    assert not missing, f'{_rel(path)}: unannotated {missing}'


@pytest.mark.parametrize('path', [p for p in LIB if not p.endswith('_build.py')], ids=_rel)
def test_library_does_not_print(path):
    tree = ast.parse(open(path).read())
    main_blocks = set()
    for node in tree.body:
        if isinstance(node, ast.If) and 'main' in ast.dump(node.test):
            main_blocks.update(id(n) for n in ast.walk(node))
    prints = [n.lineno for n in ast.walk(tree)
              if isinstance(n, ast.Call) and isinstance(n.func, ast.Name)
              and n.func.id == 'print' and id(n) not in main_blocks]
    assert not prints, f'{_rel(path)}: print() at lines {prints}'


FIRST_PARTY = {'torchgpipe_amd', 'tests', 'benchmarks', 'torchgpipe_amd_balancing'}


def _import_key(node):
    if isinstance(node, ast.Import):
        module = node.names[0].name
    else:
        module = '.' * node.level + (node.module or '')
    root = module.split('.')[0]
    if root == '__future__':
        section = 0
    elif root in FIRST_PARTY or module.startswith('.'):
        section = 3
    elif root in sys.stdlib_module_names:
        section = 1
    else:
        section = 2
    return section, module.lower()


@pytest.mark.parametrize('path', LIB, ids=_rel)
def test_import_order(path):
    tree = ast.parse(open(path).read())
    block = []
    for node in tree.body:
        if isinstance(node, (ast.Import, ast.ImportFrom)):
            block.append(node)
        elif block and not (isinstance(node, ast.Expr) and isinstance(node.value, ast.Constant)):
            break
    keys = [_import_key(n) for n in block]
    unsorted = [block[i].lineno for i in range(1, len(keys)) if keys[i] < keys[i - 1]]
    assert not unsorted, f'{_rel(path)}: imports out of isort order at lines {unsorted}'
