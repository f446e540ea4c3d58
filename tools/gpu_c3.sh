#!/bin/bash
# C3 (SAM P70, 32768 x 1024-frame calls): the RX parity tests that run the AM / SAM fronts
# (segmented 1024 / 2048-frame calls included), then the C3 line and its rocprofv3 kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-a}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_sizes.py tests/test_gpu_pipelined.py -x -q --timeout 240 --timeout-method thread > gpurun_out/c3_pytest_$tag.log 2>&1; rc=$?
tail -3 gpurun_out/c3_pytest_$tag.log
[ $rc -eq 0 ] || { tail -60 gpurun_out/c3_pytest_$tag.log; exit $rc; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c3_prof_$tag -o prof --output-format csv -- python tools/bench_configs.py --only c3 --steps 50 > gpurun_out/c3_prof_$tag.log 2>&1 || { tail -20 gpurun_out/c3_prof_$tag.log; exit 1; }
timeout -k 10 200 python tools/bench_configs.py --only c3 --steps 50 > gpurun_out/c3_lines_$tag.jsonl 2>&1 || { tail -20 gpurun_out/c3_lines_$tag.jsonl; exit 1; }
grep '^{' gpurun_out/c3_lines_$tag.jsonl
python tools/kstats.py $(find gpurun_out/c3_prof_$tag -name '*kernel_stats.csv')
