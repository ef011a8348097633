#!/bin/bash
# Heavy entities on a side-stream csr-kernel launch concurrent with the lean launch: tests + game5pl A/B + micro.
set -o pipefail
mkdir -p gpurun_out/r4tail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_game_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4tail/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r4tail/pytest.log; exit 1; }
tail -2 gpurun_out/r4tail/pytest.log
for ts in 0 768 256 2048; do
  PML_RE_TAIL_SHARE=$ts timeout -k 10 400 python -u bench_game.py --config game5pl --steps 5 --warmup 2 > gpurun_out/r4tail/g$ts.json 2> gpurun_out/r4tail/g$ts.log || { echo "game5pl $ts failed"; tail -30 gpurun_out/r4tail/g$ts.log; exit 1; }
  echo "tail share $ts: $(cut -c130-330 gpurun_out/r4tail/g$ts.json)"
  grep "sweeps (ms)" gpurun_out/r4tail/g$ts.log
done
