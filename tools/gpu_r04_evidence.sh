#!/bin/bash
# Round-4 evidence after the parity suite (tools/gpu_r04.sh): smoke, the default bench line,
# rocprofv3 kernel-trace stats (C2, north star EXACT / FMA) and PMC passes (north star EXACT /
# FMA, C2).  Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r04}
step() { echo "=== $1 ($(date +%T))"; }
step "smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step "bench (default)"
timeout -k 10 400 python bench.py > gpurun_out/bench_${tag}.json 2> gpurun_out/bench_${tag}.err || { tail -30 gpurun_out/bench_${tag}.err; exit 1; }
cat gpurun_out/bench_${tag}.json
step "rocprof kernel trace c2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2_${tag} -o prof --output-format csv -- python bench.py --steps 200 --warmup 20 --no-cpu --no-northstar > gpurun_out/prof_c2_${tag}.log 2>&1 || { tail -20 gpurun_out/prof_c2_${tag}.log; exit 1; }
step "rocprof kernel trace northstar"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ns_${tag} -o prof --output-format csv -- python bench.py --workload northstar --steps 100 --warmup 10 --no-cpu > gpurun_out/prof_ns_${tag}.log 2>&1 || { tail -20 gpurun_out/prof_ns_${tag}.log; exit 1; }
step "rocprof kernel trace northstar fma"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_nsfma_${tag} -o prof --output-format csv -- python bench.py --workload northstar --precision fma --steps 100 --warmup 10 --no-cpu > gpurun_out/prof_nsfma_${tag}.log 2>&1 || { tail -20 gpurun_out/prof_nsfma_${tag}.log; exit 1; }
step "pmc northstar"
bash tools/gpu_pmc.sh ns_${tag} --workload northstar --steps 5 --warmup 2 || exit 1
step "pmc northstar fma"
bash tools/gpu_pmc.sh nsfma_${tag} --workload northstar --precision fma --steps 5 --warmup 2 || exit 1
step "pmc c2"
bash tools/gpu_pmc.sh c2_${tag} --steps 20 --warmup 5 || exit 1
python tools/pmc_summary.py ns_${tag} > gpurun_out/pmc_northstar_${tag}.json
python tools/pmc_summary.py c2_${tag} > gpurun_out/pmc_c2_${tag}.json
python tools/pmc_summary.py nsfma_${tag} > gpurun_out/pmc_northstar_fma_${tag}.json
echo DONE
