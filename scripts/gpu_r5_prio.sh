#!/bin/bash
# Round 5: stream priority of the RE pass-path (sub) and row-space (side) streams: game5heavy and game5pl.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5prio
mkdir -p $out
python3 -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
for cfg in "game5heavy 0 0" "game5heavy -1 0" "game5pl 0 0" "game5pl 0 -1"; do
  set -- $cfg
  PML_RE_SUB_PRIORITY=$2 PML_RE_SIDE_PRIORITY=$3 timeout -k 10 500 python -u bench_game.py --config $1 --steps 3 --warmup 2 > $out/$1_$2_$3.json 2> $out/$1_$2_$3.log || { echo "bench failed"; tail -30 $out/$1_$2_$3.log; exit 1; }
  echo "$1 sub=$2 side=$3: $(grep -o '"coordinate_ms[^}]*}' $out/$1_$2_$3.json) $(grep -o 'sweeps (ms).*' $out/$1_$2_$3.log)"
done
