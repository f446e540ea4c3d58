#!/bin/bash
# Round-4 check: the full GPU parity suite, then the driver-style bench line (20 steps) and a
# longer one, each step under its own time limit; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-a}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu_$tag.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu_$tag.log
[ $rc -eq 0 ] || { tail -80 gpurun_out/pytest_gpu_$tag.log; exit $rc; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench20_$tag.json 2> gpurun_out/bench20_$tag.err || { tail -30 gpurun_out/bench20_$tag.err; exit 1; }
cat gpurun_out/bench20_$tag.json
