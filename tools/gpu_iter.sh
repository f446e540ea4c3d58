#!/bin/bash
# Iteration loop on one GPU box: parity suite, then a short bench (no CPU leg).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-iter}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_${tag}.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_${tag}.log
[ $rc -eq 0 ] || { tail -60 gpurun_out/pytest_gpu_${tag}.log; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu --steps 300 --warmup 20 > gpurun_out/bench_${tag}.json 2> gpurun_out/bench_${tag}.err || { tail -30 gpurun_out/bench_${tag}.err; exit 1; }
cat gpurun_out/bench_${tag}.json
