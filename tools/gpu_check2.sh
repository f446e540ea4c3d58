#!/bin/bash
# Parity suite, smoke and the default bench line (with the box's CPU facts), each step time-limited.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-cur}
echo "nproc=$(nproc) affinity=$(python -c 'import os;print(len(os.sched_getaffinity(0)))') OMP=$OMP_NUM_THREADS $(grep -m1 'model name' /proc/cpuinfo)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_${tag}.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu_${tag}.log
[ $rc -eq 0 ] || { tail -80 gpurun_out/pytest_gpu_${tag}.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
timeout -k 10 400 python bench.py --steps 20 > gpurun_out/bench20_${tag}.json 2> gpurun_out/bench20_${tag}.err || { tail -30 gpurun_out/bench20_${tag}.err; exit 1; }
cat gpurun_out/bench20_${tag}.json
