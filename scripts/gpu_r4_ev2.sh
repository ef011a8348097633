#!/bin/bash
# LDS add-order probe test, then the 2-rank gloo rehearsal of bench.py on one GPU (routing with the GPU permutation
# and the host-bypassing kept segment).
set -o pipefail
mkdir -p gpurun_out/r4ev2
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -s --timeout 120 --timeout-method thread -k "lds_same_address" > gpurun_out/r4ev2/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r4ev2/pytest.log; exit 1; }
tail -2 gpurun_out/r4ev2/pytest.log
PML_DIST_BACKEND=gloo timeout -k 10 1000 python -u bench.py --gpus 2 --rehearsal --rows-per-gpu 4000000 --steps 3 --warmup 2 > gpurun_out/r4ev2/rehearsal.json 2> gpurun_out/r4ev2/rehearsal.log || { echo "rehearsal failed"; tail -30 gpurun_out/r4ev2/rehearsal.log; exit 1; }
grep -v Gloo gpurun_out/r4ev2/rehearsal.json | cut -c1-3500
