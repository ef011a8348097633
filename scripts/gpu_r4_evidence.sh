#!/bin/bash
# Round 4 evidence runs: (1) Avro -> device-layout ingest at 1e9 non-zeros (16 threads = the box's CPU share),
# (2) the 2-rank gloo rehearsal of bench.py on one GPU (GLM headline at 4M rows/rank + game5pl entity-sharded,
# 1.25M entities per rank, with the per-phase routing times).
set -o pipefail
mkdir -p gpurun_out/r4ev
export TMPDIR=/tmp
PML_AVRO_THREADS=16 timeout -k 10 900 python -u scripts/ingest_bench.py --records 10000000 --nnz 100 --files 64 --dir /tmp/pml_ingest --device cuda --out gpurun_out/r4ev/ingest_1e9.json > gpurun_out/r4ev/ingest.log 2>&1 || { echo "ingest failed"; tail -20 gpurun_out/r4ev/ingest.log; exit 1; }
tail -3 gpurun_out/r4ev/ingest.log
rm -rf /tmp/pml_ingest
PML_DIST_BACKEND=gloo timeout -k 10 1000 python -u bench.py --gpus 2 --rehearsal --rows-per-gpu 4000000 --steps 3 --warmup 2 > gpurun_out/r4ev/rehearsal.json 2> gpurun_out/r4ev/rehearsal.log || { echo "rehearsal failed"; tail -30 gpurun_out/r4ev/rehearsal.log; exit 1; }
grep -v Gloo gpurun_out/r4ev/rehearsal.json | cut -c1-3000
grep -E "routing|route" gpurun_out/r4ev/rehearsal.log | head -8
