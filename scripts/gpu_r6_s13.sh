#!/bin/bash
# Round 6 step 13: driver-contract bench record (GAME metric first), CLI one-shot at scale, fresh-process one-shot.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6s13
mkdir -p $out
timeout -k 10 700 python -u bench.py > $out/bench.json 2> $out/bench.log || { echo "bench failed"; tail -30 $out/bench.log; exit 1; }
python3 -c "
import json; d=json.load(open('$out/bench.json'))
print({k: d[k] for k in ('value','ms_per_step')})
print({k: (round(v,2) if isinstance(v,float) else v) for k,v in d.items() if k.startswith('game5pl') and ('ms' in k or '_s' in k)})
"
PML_SYNC_TIMED=1 timeout -k 10 600 python -u scripts/cli_oneshot.py --records 10000000 --nnz 30 --entities 500000 --dir /tmp/pml_cli --out $out/cli.json > $out/cli.log 2>&1 || { echo "cli failed"; tail -30 $out/cli.log; exit 1; }
grep -E "Avro read|Read training|Fit models|Save models" $out/cli.log
timeout -k 10 300 python -u scripts/oneshot_profile.py --precisions bf16,f64 --json $out/nosync.json > $out/nosync.md 2> $out/nosync.log || { echo "oneshot failed"; tail -30 $out/nosync.log; exit 1; }
grep -E "warm-up" $out/nosync.md
