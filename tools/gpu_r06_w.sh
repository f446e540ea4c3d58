#!/bin/bash
# Round 6 (w): the driver's bench command three times against the C2-only line (no CPU / north-star
# legs) three times, interleaved: does the full command's C2 number differ from the C2-only line?
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06w}
for i in 1 2 3; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/full_$tag.json 2> gpurun_out/full_$tag.err || { tail -30 gpurun_out/full_$tag.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('full', d['ms_per_step'], d['value'], d['handoff_timeouts'])" gpurun_out/full_$tag.json | tee -a gpurun_out/w_$tag.txt
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-northstar > gpurun_out/c2_$tag.json 2> gpurun_out/c2_$tag.err || { tail -30 gpurun_out/c2_$tag.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('c2only', d['ms_per_step'], d['value'], d['handoff_timeouts'])" gpurun_out/c2_$tag.json | tee -a gpurun_out/w_$tag.txt
done
