#!/bin/bash
# Round 6 (fb): C2 in mode 3 with 8 (default) and 16 front outputs per lane, 20 x3 / 1000, two rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06fb}
for round in 1 2; do
  for fb in 8 16; do
    for steps in 20 20 20 1000; do
      timeout -k 10 200 python bench.py --steps $steps --warmup 5 --no-cpu --no-northstar --front-block $fb > gpurun_out/fb_$tag.json 2> gpurun_out/fb_$tag.err || { tail -20 gpurun_out/fb_$tag.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['ms_per_step'], d['value'], d['handoff_timeouts'], d['chain']['kernel_ms'])" gpurun_out/fb_$tag.json $fb $steps | tee -a gpurun_out/fb_$tag.txt
    done
  done
done
