#!/bin/bash
# The TX chain: its parity tests (bit-exact, pipelined, FMA precision), the C4 SSB-TX lines in
# EXACT and FMA precision, then a rocprofv3 kernel trace of both lines (tx_voice2 / tx_iq times).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-a}
timeout -k 10 400 python -u -m pytest tests/test_gpu_tx.py tests/test_gpu_tx_pipelined.py tests/test_gpu_tx_precision.py -x -q -s --timeout 200 --timeout-method thread > gpurun_out/tx_pytest_$tag.log 2>&1; rc=$?
grep -E "tx fma|passed|failed" gpurun_out/tx_pytest_$tag.log | tail -20
[ $rc -eq 0 ] || { tail -60 gpurun_out/tx_pytest_$tag.log; exit $rc; }
timeout -k 10 200 python tools/bench_configs.py --only c4tx,c4txfma --steps 50 > gpurun_out/tx_lines_$tag.jsonl 2>&1 || { tail -20 gpurun_out/tx_lines_$tag.jsonl; exit 1; }
grep '^{' gpurun_out/tx_lines_$tag.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/tx_prof_$tag -o prof --output-format csv -- python tools/bench_configs.py --only c4tx,c4txfma --steps 50 > gpurun_out/tx_prof_$tag.log 2>&1 || { tail -20 gpurun_out/tx_prof_$tag.log; exit 1; }
python tools/kstats.py $(find gpurun_out/tx_prof_$tag -name '*kernel_stats.csv')
