#!/bin/bash
# Round 6 step 38: GAME GPU tests incl. the lazy pass-layout regression test.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6s38
mkdir -p $out
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_game_gpu.py > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
