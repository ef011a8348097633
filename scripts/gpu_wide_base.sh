#!/bin/bash
# Wide-round key bases (ops/tiled.py TLFwdChunk): kernel parity tests, headline bench (1M features: no bases, the
# extra scalar base load per round must cost nothing), OWL-QN at 10M features with bases (1024-row blocks) and
# without (256-row blocks).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "wide_round or value_grad_parity or tl_multi or margins or hessian_parity" --timeout 200 --timeout-method thread > gpurun_out/pytest_wide.log 2>&1 || { tail -30 gpurun_out/pytest_wide.log; exit 1; }
tail -1 gpurun_out/pytest_wide.log
timeout -k 10 300 python bench.py --game off > gpurun_out/hl_wide.json 2> gpurun_out/hl_wide.log || exit 1
cut -c150-260 gpurun_out/hl_wide.json
timeout -k 10 300 python bench.py --config owlqn --game off > gpurun_out/owlqn_wide.json 2> gpurun_out/owlqn_wide.log || exit 1
cut -c150-260 gpurun_out/owlqn_wide.json
PML_TL_WIDE_BASE=0 timeout -k 10 300 python bench.py --config owlqn --game off > gpurun_out/owlqn_nowide.json 2> gpurun_out/owlqn_nowide.log || exit 1
cut -c150-260 gpurun_out/owlqn_nowide.json
