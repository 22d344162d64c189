"""Small AST linter run as a test (the reference runs ESLint from mocha: test/eslint.js:1-30,
config ``.eslintrc.yaml`` = standard). No flake8/ruff in the image, so the checks that matter
are implemented here:

  E999 syntax error          F401 unused import           E501 line too long
  W191 tab indentation       W291 trailing whitespace     E722 bare ``except:``
  B006 mutable default arg   F811 redefined function in the same scope
  A001 ``asyncio.gather`` without ``return_exceptions=True`` (its failure leaves the
       sibling awaitables running: use ``utils.aio.gather_strict``)

Settings live in ``pyproject.toml`` under ``[tool.stager-lint]``; ``# noqa`` on a line skips it.
Usage: ``python -m downloader_amd.utils.lint [paths...]``.
"""
from __future__ import annotations

import ast
import os
import sys
from dataclasses import dataclass
from typing import Iterable, List, Sequence, Set

MAX_LINE = 110


@dataclass
class Finding:
    path: str
    line: int
    code: str
    msg: str

    def __str__(self) -> str:
        return f"{self.path}:{self.line}: {self.code} {self.msg}"


def _names_used(tree: ast.AST) -> Set[str]:
    used: Set[str] = set()
    for n in ast.walk(tree):
        if isinstance(n, ast.Name):
            used.add(n.id)
        elif isinstance(n, ast.Attribute):
            base = n
            while isinstance(base, ast.Attribute):
                base = base.value
            if isinstance(base, ast.Name):
                used.add(base.id)
        elif isinstance(n, ast.Constant) and isinstance(n.value, str):
            # names referenced from string annotations / __all__
            for tok in n.value.replace("[", " ").replace("]", " ").replace(",", " ").split():
                used.add(tok.split(".")[0].strip("'\""))
    return used


def lint_source(path: str, src: str, max_line: int = MAX_LINE) -> List[Finding]:
    out: List[Finding] = []
    lines = src.splitlines()
    noqa = {i + 1 for i, l in enumerate(lines) if "# noqa" in l}
    try:
        tree = ast.parse(src, filename=path)
    except SyntaxError as e:
        return [Finding(path, e.lineno or 0, "E999", f"syntax error: {e.msg}")]
    for i, l in enumerate(lines, 1):
        if i in noqa:
            continue
        if len(l) > max_line:
            out.append(Finding(path, i, "E501", f"line too long ({len(l)} > {max_line})"))
        if l.startswith("\t"):
            out.append(Finding(path, i, "W191", "tab indentation"))
        if l.rstrip() != l:
            out.append(Finding(path, i, "W291", "trailing whitespace"))
    is_init = os.path.basename(path) == "__init__.py"
    used = _names_used(tree)
    for n in ast.walk(tree):
        if isinstance(n, ast.ExceptHandler) and n.type is None and n.lineno not in noqa:
            out.append(Finding(path, n.lineno, "E722", "bare except"))
        if isinstance(n, ast.Call) and isinstance(n.func, ast.Attribute) and \
                n.func.attr == "gather" and isinstance(n.func.value, ast.Name) and \
                n.func.value.id == "asyncio" and n.lineno not in noqa and not any(
                    k.arg == "return_exceptions" for k in n.keywords):
            out.append(Finding(path, n.lineno, "A001", "asyncio.gather leaves siblings running "
                                                       "on failure: use utils.aio.gather_strict"))
        if isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef)):
            for d in n.args.defaults + n.args.kw_defaults:
                if isinstance(d, (ast.List, ast.Dict, ast.Set)) and n.lineno not in noqa:
                    out.append(Finding(path, n.lineno, "B006",
                                       f"mutable default argument in {n.name}()"))
        if isinstance(n, (ast.Module, ast.ClassDef)):
            seen = {}
            for st in n.body:
                if isinstance(st, (ast.FunctionDef, ast.AsyncFunctionDef)):
                    decorated = bool(st.decorator_list)
                    if st.name in seen and not decorated and st.lineno not in noqa:
                        out.append(Finding(path, st.lineno, "F811",
                                           f"redefinition of {st.name} from line {seen[st.name]}"))
                    seen[st.name] = st.lineno
    if not is_init:
        for n in tree.body if isinstance(tree, ast.Module) else []:
            if isinstance(n, (ast.Import, ast.ImportFrom)) and n.lineno not in noqa:
                if isinstance(n, ast.ImportFrom) and n.module == "__future__":
                    continue
                for a in n.names:
                    name = (a.asname or a.name).split(".")[0]
                    if name != "*" and name not in used:
                        out.append(Finding(path, n.lineno, "F401", f"'{a.name}' imported but unused"))
    return out


def iter_py(paths: Sequence[str]) -> Iterable[str]:
    for p in paths:
        if os.path.isfile(p) and p.endswith(".py"):
            yield p
        elif os.path.isdir(p):
            for dp, dns, fns in os.walk(p):
                dns[:] = [d for d in dns if not d.startswith((".", "__pycache__", "build"))]
                for fn in sorted(fns):
                    if fn.endswith(".py"):
                        yield os.path.join(dp, fn)


def lint_paths(paths: Sequence[str], max_line: int = MAX_LINE) -> List[Finding]:
    out: List[Finding] = []
    for p in iter_py(paths):
        with open(p, "r", encoding="utf-8") as f:
            out += lint_source(p, f.read(), max_line)
    return out


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv) or ["downloader_amd", "tests", "bench.py"]
    found = lint_paths(argv)
    for f in found:
        print(f)
    return 1 if found else 0


if __name__ == "__main__":
    sys.exit(main())
