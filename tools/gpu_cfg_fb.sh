#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for fb in 8 16 0; do
  timeout -k 10 300 python tools/bench_configs.py --only c3,c5 --front-block $fb > gpurun_out/fb_$fb.jsonl 2> gpurun_out/fb_$fb.err || { tail gpurun_out/fb_$fb.err; exit 1; }
  python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print('fb', sys.argv[2], d['workload'][:20], d['ms_per_call'], d.get('kernel_ms'), d['hbm_frac'], d['finite'])" gpurun_out/fb_$fb.jsonl $fb
done
bash tools/gpu_configs.sh r03c c3,c3spec,c4fm,c4tx,c5,c5fir
