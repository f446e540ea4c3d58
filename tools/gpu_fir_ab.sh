#!/bin/bash
# A/B of the batched FIR's waves per workgroup (uhsdr_fir_set_waves): the parity tests (which
# cover 1, 2 and 4 waves), then the C5 FIR config lines at each count
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fir.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fir_ab_pytest.log 2>&1 || { tail -30 gpurun_out/fir_ab_pytest.log; exit 1; }
tail -1 gpurun_out/fir_ab_pytest.log
for wv in 4 2 1; do
  timeout -k 10 200 python tools/bench_configs.py --only c5fir --fir-waves $wv > gpurun_out/fir_ab_$wv.jsonl 2> gpurun_out/fir_ab_$wv.err || { tail -20 gpurun_out/fir_ab_$wv.err; exit 1; }
  cut -c1-300 gpurun_out/fir_ab_$wv.jsonl
done
