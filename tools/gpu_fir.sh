#!/bin/bash
# batched FIR check: its parity tests, then the C5 FIR config lines (EXACT and MFMA)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fir.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fir_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/fir_pytest.log
[ $rc -eq 0 ] || { grep -m5 -B5 -A30 "Error\|FAIL" gpurun_out/fir_pytest.log | head -80; exit $rc; }
timeout -k 10 200 python tools/bench_configs.py --only c5fir > gpurun_out/fir_cfg.jsonl 2> gpurun_out/fir_cfg.err || { tail -20 gpurun_out/fir_cfg.err; exit 1; }
cut -c1-400 gpurun_out/fir_cfg.jsonl
