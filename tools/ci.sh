#!/usr/bin/env bash
# Continuous-integration entry point (the reference's .travis.yml runs
# install -> pycodestyle / flake8 -> pytest -> docs; here):
#   1. build every native library for gfx950 (hipcc cross-compiles, no GPU);
#   2. lint (tools/lint.sh: flake8 / clang-format when present + tools/lint.py);
#   3. CPU test suite (pytest -m "not gpu", gloo for the multi-process tests);
#   4. docs: every file the README links exists;
#   5. with --gpu on an MI355X host: the GPU test suite and smoke().
# Every stage has its own time limit; the first failure ends the run.
set -euo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
stage() { echo "== $1"; }
stage build
timeout -k 10 1800 python -c "import __graft_entry__ as g; g.build()"
stage lint
timeout -k 10 600 bash tools/lint.sh
stage cpu-tests
timeout -k 10 2400 python -m pytest tests -x -q -m "not gpu" -p no:cacheprovider
stage docs
python - <<'PY'
import re, os, sys
bad = [m for m in re.findall(r'\]\(([^)#]+)\)', open('README.md').read())
       if not m.startswith('http') and not os.path.exists(m)]
if bad:
    sys.exit('README links to missing files: %s' % bad)
PY
if [ "${1:-}" = "--gpu" ]; then
  stage gpu-tests
  timeout -k 10 1200 python -u -m pytest tests -x -v -m gpu --timeout 300 \
    --timeout-method thread
  stage smoke
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
echo "ci ok"
