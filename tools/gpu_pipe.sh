#!/bin/bash
# Pipelined-mode check: its parity tests, then C2 and north-star bench lines with and without
# the front/back overlap (no CPU leg).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipelined.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_pipe.log 2>&1; rc=$?
tail -12 gpurun_out/pytest_pipe.log
[ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; tail -60 gpurun_out/pytest_pipe.log; exit $rc; }
for m in "" "--serial"; do
  tag=${m:-pipe}; tag=${tag#--}
  timeout -k 10 300 python bench.py --steps 1000 --warmup 50 --no-cpu --no-northstar $m > gpurun_out/c2_$tag.json 2> gpurun_out/c2_$tag.err || { cat gpurun_out/c2_$tag.err; exit 1; }
  cat gpurun_out/c2_$tag.json
  timeout -k 10 300 python bench.py --workload northstar --steps 20 --warmup 3 --no-cpu $m > gpurun_out/ns_$tag.json 2> gpurun_out/ns_$tag.err || { cat gpurun_out/ns_$tag.err; exit 1; }
  cat gpurun_out/ns_$tag.json
done
