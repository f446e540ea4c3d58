#!/bin/bash
# FMA-precision check: its tolerance tests, the pipelined tests, then bench lines
# (C2 pipelined / serial, north star exact / fma; no CPU leg).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_fma.py tests/test_gpu_pipelined.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_fma.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|passed|failed" gpurun_out/pytest_fma.log | tail -45
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest rc=$rc"; exit $rc; }
run() { tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu "$@" > gpurun_out/b_$tag.json 2> gpurun_out/b_$tag.err || { cat gpurun_out/b_$tag.err; exit 1; }; cat gpurun_out/b_$tag.json; }
run c2_pipe --steps 1000 --warmup 50 --no-northstar
run c2_serial --steps 1000 --warmup 50 --no-northstar --serial
run ns_exact --workload northstar --steps 20 --warmup 3
run ns_fma --workload northstar --steps 20 --warmup 3 --precision fma
run c2_fma --steps 1000 --warmup 50 --no-northstar --precision fma
