#!/bin/bash
# Iteration on one GPU box: the parity suite, then north-star (1M x 64) and C2 bench lines
# and a kernel-trace summary of the north-star run.  Usage: tools/gpu_ns.sh <tag> [--no-tests]
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-ns}
if [ "$2" != "--no-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${tag}.log 2>&1; rc=$?
  tail -3 gpurun_out/pytest_${tag}.log
  [ $rc -eq 0 ] || { tail -60 gpurun_out/pytest_${tag}.log; exit $rc; }
fi
timeout -k 10 300 python bench.py --workload northstar --steps 20 --warmup 3 --no-cpu > gpurun_out/ns_${tag}.json 2> gpurun_out/ns_${tag}.err || { tail -30 gpurun_out/ns_${tag}.err; exit 1; }
cat gpurun_out/ns_${tag}.json
timeout -k 10 300 python bench.py --steps 1000 --warmup 50 --no-cpu --no-northstar > gpurun_out/c2_${tag}.json 2> gpurun_out/c2_${tag}.err || { tail -30 gpurun_out/c2_${tag}.err; exit 1; }
cat gpurun_out/c2_${tag}.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ns_${tag} -o prof --output-format csv -- python bench.py --workload northstar --steps 20 --warmup 3 --no-cpu > gpurun_out/prof_ns_${tag}.log 2>&1 || { tail -20 gpurun_out/prof_ns_${tag}.log; exit 1; }
python tools/kstats.py gpurun_out/prof_ns_${tag}/prof_kernel_stats.csv
