#!/bin/bash
# C5 FIR lines (EXACT and MFMA) for library builds: each argument "label|ENV=..."
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in "$@"; do
  IFS='|' read label envs <<< "$v"
  env $envs timeout -k 10 200 python tools/bench_configs.py --only c5fir > gpurun_out/firlib_$label.jsonl 2> gpurun_out/firlib_$label.err || { tail -20 gpurun_out/firlib_$label.err; exit 1; }
  python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(sys.argv[2], d['workload'][-40:], d['ms_per_call'], d.get('mfma_tflops_issued'))" gpurun_out/firlib_$label.jsonl $label
done
