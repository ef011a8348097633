#!/bin/bash
# Waves per workgroup of the TL kernels on the sparse GAME FE shard (experiment build: PML_GLM_LIB = libpml_glm_abl.so).
set -o pipefail
out=gpurun_out/${1:-fewaves}
mkdir -p $out
export TMPDIR=/tmp
export PML_GLM_LIB=$GRAFT_REPO_ROOT/photon_ml_amd/ops/_lib/libpml_glm_abl.so
run() {  # tag prec env...
  local tag=$1 prec=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench_game.py --config game5pl --precision $prec --steps 3 --warmup 2 > $out/g_$tag.json 2> $out/g_$tag.log || { echo "$tag failed"; tail -20 $out/g_$tag.log; return 1; }
  echo "$tag: $(grep -o '"coordinate_ms[^}]*}' $out/g_$tag.json)"
}
run bf16_t4 bf16 PML_TL_WAVES_T=4 && run bf16_t2 bf16 PML_TL_WAVES_T=2 && run bf16_f4 bf16 PML_TL_WAVES=4 && \
run f64_t4 f64 PML_TL_WAVES_T=4 && run f64_t2 f64 PML_TL_WAVES_T=2 && run bf16_t2b bf16 PML_TL_WAVES_T=2 && run bf16_t4b bf16 PML_TL_WAVES_T=4
