#!/bin/bash
# One GPU session: parity tests, smoke, short bench, kernel-trace profile.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "=== $1 ($(date +%T))"; }
step "rocminfo"; (rocm-smi --showproductname 2>/dev/null | head -8) || true
step "pytest gpu"
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest gpu failed rc=$rc"; tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
step "smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step "bench c2"
timeout -k 10 300 python bench.py --steps 500 --warmup 50 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { cat gpurun_out/bench_c2.err; exit 1; }
cat gpurun_out/bench_c2.json
step "bench northstar"
timeout -k 10 400 python bench.py --workload northstar --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_ns.json 2> gpurun_out/bench_ns.err || { cat gpurun_out/bench_ns.err; exit 1; }
cat gpurun_out/bench_ns.json
step "rocprof kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o prof --output-format csv -- python bench.py --steps 200 --warmup 20 --no-cpu > gpurun_out/prof_c2.log 2>&1 || { tail -20 gpurun_out/prof_c2.log; exit 1; }
find gpurun_out/prof_c2 -name "*stats*" | head
echo DONE
