"""Lint as a test (the reference runs ESLint from mocha, test/eslint.js:1-30)."""
from __future__ import annotations

import os

from downloader_amd.utils.lint import lint_paths, lint_source

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_repository_is_lint_clean():
    paths = [os.path.join(REPO, p) for p in ("downloader_amd", "tests", "bench.py",
                                               "__graft_entry__.py")]
    found = lint_paths(paths)
    assert not found, "\n".join(str(f) for f in found)


def test_linter_catches_problems():
    src = "import os\nimport sys\n\ndef f(x=[]):\n    try:\n        pass\n    except:\n        pass\n" \
          "    return sys.argv\n"
    codes = sorted(f.code for f in lint_source("x.py", src))
    assert codes == ["B006", "E722", "F401"]
    assert [f.code for f in lint_source("y.py", "def (:\n")] == ["E999"]


def test_a001_flags_gather_that_leaves_siblings_running():
    bad = "import asyncio\n\n\nasync def f(a, b):\n    await asyncio.gather(a, b)\n"
    ok = ("import asyncio\n\n\nasync def f(a, b):\n"
          "    await asyncio.gather(a, b, return_exceptions=True)\n")
    assert [f.code for f in lint_source("a.py", bad)] == ["A001"]
    assert lint_source("b.py", ok) == []
