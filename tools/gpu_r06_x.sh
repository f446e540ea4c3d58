#!/bin/bash
# Round 6 (x): the main build, C2 with the device hand-off against the persistent back end,
# interleaved on one box (20 / 20 / 1000 steps, two rounds).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06x}
for round in 1 2; do
  for m in device persistent; do
    for steps in 20 20 1000; do
      timeout -k 10 200 python bench.py --steps $steps --warmup 5 --no-cpu --no-northstar --handoff $m > gpurun_out/x_$tag.json 2> gpurun_out/x_$tag.err || { tail -20 gpurun_out/x_$tag.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['ms_per_step'], d['value'], d['handoff_timeouts'])" gpurun_out/x_$tag.json $m $steps | tee -a gpurun_out/x_$tag.txt
    done
  done
done
