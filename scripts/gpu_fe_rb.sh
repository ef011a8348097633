#!/bin/bash
# Forward row-block bits on the sparse FE shard (transpose tiles by the shard heuristic), bf16 and fp64.
set -o pipefail
out=gpurun_out/${1:-ferb}
mkdir -p $out
export TMPDIR=/tmp
run() {  # tag prec env...
  local tag=$1 prec=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench_game.py --config game5pl --precision $prec --steps 3 --warmup 2 > $out/g_$tag.json 2> $out/g_$tag.log || { echo "$tag failed"; tail -20 $out/g_$tag.log; return 1; }
  echo "$tag: $(grep -o '"coordinate_ms[^}]*}' $out/g_$tag.json)"
}
run bf16_rb10 bf16 PML_TL_RBITS=10 && run bf16_rb11 bf16 PML_TL_RBITS=11 && run f64_rb10 f64 PML_TL_RBITS=10 && \
run f64_rb11 f64 PML_TL_RBITS=11 && run bf16_rb11b bf16 PML_TL_RBITS=11 && run f64_rb11b f64 PML_TL_RBITS=11 && run bf16_rb10b bf16 PML_TL_RBITS=10
