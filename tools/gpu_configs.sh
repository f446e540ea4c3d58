#!/bin/bash
# Evidence for the non-headline configs (tools/bench_configs.py): throughput lines, one
# rocprofv3 kernel-trace summary, and PMC passes (tools/gpu_pmc_cmd.sh) per config.
# Usage: tools/gpu_configs.sh <tag> [configs, default c3,c3spec,c4fm,c4tx,c5,c5fir]
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-cfg}
cfgs=${2:-c3,c3spec,c4fm,c4tx,c5,c5fir}
echo "=== bench_configs ($(date +%T))"
timeout -k 10 400 python tools/bench_configs.py --only $cfgs > gpurun_out/configs_${tag}.jsonl 2> gpurun_out/configs_${tag}.err || { tail -20 gpurun_out/configs_${tag}.err; exit 1; }
cat gpurun_out/configs_${tag}.jsonl
for c in ${cfgs//,/ }; do
  echo "=== kernel trace $c ($(date +%T))"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_${tag}_$c -o prof --output-format csv -- python tools/bench_configs.py --only $c --steps 20 --warmup 3 > gpurun_out/kt_${tag}_$c.log 2>&1 || { tail -20 gpurun_out/kt_${tag}_$c.log; exit 1; }
  python tools/kstats.py gpurun_out/kt_${tag}_$c/prof_kernel_stats.csv
  echo "=== pmc $c ($(date +%T))"
  bash tools/gpu_pmc_cmd.sh ${tag}_$c tools/bench_configs.py --only $c --steps 5 --warmup 2 > gpurun_out/pmc_${tag}_$c.json 2> gpurun_out/pmc_${tag}_$c.err || { tail -20 gpurun_out/pmc_${tag}_$c.json; exit 1; }
done
echo DONE
