#!/usr/bin/env bash
# Repository lint: flake8 + clang-format (dry run) when installed, plus the
# self-contained checker (line length, whitespace, unused imports, and the
# MI355X-only rules for csrc/) which needs nothing but Python.
set -euo pipefail
cd "$(dirname "$0")/.."
rc=0
if command -v flake8 >/dev/null 2>&1; then
  flake8 deep_graph_matching_consensus_amd tests tools examples bench.py || rc=1
fi
if command -v clang-format >/dev/null 2>&1; then
  find csrc -name '*.hip' -o -name '*.cpp' -o -name '*.h' |
    xargs clang-format --dry-run -Werror || rc=1
fi
python tools/lint.py || rc=1
exit $rc
