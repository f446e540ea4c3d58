#!/bin/bash
# C2 per-step time against the timed steps K and warm-up W (fixed overhead vs slope), device hand-off.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for kw in 20:5 20:200 40:5 80:5 160:5 1000:50 20:5 20:200; do
  K=${kw%%:*}; W=${kw#*:}
  timeout -k 10 200 python bench.py --steps $K --warmup $W --no-cpu --no-northstar > gpurun_out/kw_$K_$W.json 2> gpurun_out/kw.err || { tail -20 gpurun_out/kw.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('K', $K, 'W', $W, d['ms_per_step'], round(d['ms_per_step']*$K*1e3,1), 'us total')" gpurun_out/kw_$K_$W.json
done
