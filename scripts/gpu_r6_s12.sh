#!/bin/bash
# Round 6 step 12: GPU tests of the touched paths, the CLI one-shot at scale, a fresh driver-contract bench record.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6s12
mkdir -p $out
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_lbfgs_plan_gpu.py tests/test_kernels_gpu.py tests/test_fastpath_parity_gpu.py tests/test_cli_gpu.py > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
PML_SYNC_TIMED=1 timeout -k 10 900 python -u scripts/cli_oneshot.py --records 10000000 --nnz 30 --entities 500000 --dir /tmp/pml_cli --out $out/cli.json > $out/cli.log 2>&1 || { echo "cli failed"; tail -30 $out/cli.log; exit 1; }
grep -E "Avro read|Read training|Fit models|Save models|Coordinate descent" $out/cli.log
python3 -c "import json; d=json.load(open('$out/cli.json')); print('cli total', d['driver_total_s'], 'model MiB', d['model_mib'], 'entity ids', d['phases_s'].get('RE dataset: entity ids'))"
timeout -k 10 900 python -u bench.py > $out/bench.json 2> $out/bench.log || { echo "bench failed"; tail -30 $out/bench.log; exit 1; }
python3 -c "
import json; d=json.load(open('$out/bench.json'))
print({k: d[k] for k in ('value','ms_per_step')})
print({k: (round(v,2) if isinstance(v,float) else v) for k,v in d.items() if k.startswith('game5pl') and ('ms' in k or '_s' in k)})
"
