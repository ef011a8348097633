#!/bin/bash
# Round 6 step 9: the CLI one-shot at scale (Avro -> game-training -> saved model) after the host-path fixes
# (sort-based vocabulary map, reader id factorisation, uncompressed byte-sized model blocks, O(n) model codes).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6s9
mkdir -p $out
PML_SYNC_TIMED=1 timeout -k 10 900 python -u scripts/cli_oneshot.py --records 10000000 --nnz 30 --entities 500000 --dir /tmp/pml_cli --out $out/cli.json > $out/cli.log 2>&1 || { echo "cli failed"; tail -30 $out/cli.log; exit 1; }
grep -E "Avro read|Read training|entity ids|Fit models|Save models|Coordinate descent|Update coordinate" $out/cli.log
python3 -c "import json; d=json.load(open('$out/cli.json')); print('total', d['driver_total_s'], 'model MiB', d['model_mib'])"
