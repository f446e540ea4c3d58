#!/bin/bash
# RX config lines at front block 8 vs 16
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for fb in 8 16 8; do
  timeout -k 10 300 python tools/bench_configs.py --only c3,c4fm,c5 --front-block $fb > gpurun_out/e18_$fb.jsonl 2> gpurun_out/e18_$fb.err || { tail -20 gpurun_out/e18_$fb.err; exit 1; }
  python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(sys.argv[2], d['workload'][:30], d['ms_per_call'], d.get('kernel_ms'))" gpurun_out/e18_$fb.jsonl $fb
done
