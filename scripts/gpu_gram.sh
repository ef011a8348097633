#!/bin/bash
# MFMA Gram kernel: kernel / optimizer GPU tests, microbenchmark, GAME FE coordinate, headline.
set -o pipefail
out=gpurun_out/${1:-gram}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_rccl_gpu.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 120 python -u scripts/gram_mfma_bench.py > $out/micro.log 2>&1 || { echo "micro failed"; tail -20 $out/micro.log; exit 1; }
cat $out/micro.log
timeout -k 10 300 python -u bench_game.py --config game5pl --steps 3 --warmup 2 > $out/g.json 2> $out/g.log || { echo "game failed"; tail -20 $out/g.log; exit 1; }
grep -o '"coordinate_ms[^}]*}' $out/g.json
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --game off > $out/h.json 2> $out/h.log || { echo "hl failed"; tail -20 $out/h.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $out/h.json
