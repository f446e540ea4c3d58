#!/bin/bash
# Quick GPU iteration: parity tests, C2 and north-star bench lines (no CPU leg).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest gpu failed rc=$rc"; tail -60 gpurun_out/pytest_gpu.log; exit $rc; }
timeout -k 10 300 python bench.py --steps 500 --warmup 50 --no-cpu > gpurun_out/q_c2.json 2> gpurun_out/q_c2.err || { cat gpurun_out/q_c2.err; exit 1; }
cat gpurun_out/q_c2.json
timeout -k 10 300 python bench.py --workload northstar --steps 20 --warmup 3 --no-cpu > gpurun_out/q_ns.json 2> gpurun_out/q_ns.err || { cat gpurun_out/q_ns.err; exit 1; }
cat gpurun_out/q_ns.json
