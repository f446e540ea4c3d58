#!/bin/bash
# A/B of the batched FIR's waves per workgroup (UHSDR_FIR_WAVES): parity tests under each,
# then the C5 FIR config lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for wv in 4 2 1; do
  UHSDR_FIR_WAVES=$wv timeout -k 10 300 python -u -m pytest tests/test_gpu_fir.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fir_ab_pytest_$wv.log 2>&1 || { tail -30 gpurun_out/fir_ab_pytest_$wv.log; exit 1; }
  echo "waves=$wv $(tail -1 gpurun_out/fir_ab_pytest_$wv.log)"
  UHSDR_FIR_WAVES=$wv timeout -k 10 200 python tools/bench_configs.py --only c5fir > gpurun_out/fir_ab_$wv.jsonl 2> gpurun_out/fir_ab_$wv.err || { tail -20 gpurun_out/fir_ab_$wv.err; exit 1; }
  cut -c1-300 gpurun_out/fir_ab_$wv.jsonl
done
