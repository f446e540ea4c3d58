#!/bin/bash
# Round 6 (s): instruction-cache counters of the C2 kernels (one --pmc pass, SQ block only; the
# bench's device hand-off mode, 20 steps).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06s}
mkdir -p gpurun_out/pmc_$tag
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_$tag/p0 -o pmc -- python bench.py --no-cpu --no-northstar --steps 20 --warmup 5 > gpurun_out/pmc_$tag/p0.log 2>&1 || { tail -20 gpurun_out/pmc_$tag/p0.log; exit 1; }
python tools/pmc_summary.py $tag > gpurun_out/pmc_$tag.json && cat gpurun_out/pmc_$tag.json
