#!/bin/bash
# Round 6 (y): the main build against the P48-only variant build of the same sources (tools/isa
# variant table), C2 persistent back end, 20 / 20 / 1000 steps, two rounds on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06y}
for round in 1 2; do
  for lib in uhsdr_amd/lib/libuhsdr_amd.so uhsdr_amd/lib/variants/libuhsdr_amd_pers.so; do
    for steps in 20 20 1000; do
      UHSDR_LIB=$lib timeout -k 10 200 python bench.py --steps $steps --warmup 5 --no-cpu --no-northstar > gpurun_out/y_$tag.json 2> gpurun_out/y_$tag.err || { tail -20 gpurun_out/y_$tag.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['ms_per_step'], d['value'], d['handoff_timeouts'])" gpurun_out/y_$tag.json $(basename $lib .so) $steps | tee -a gpurun_out/y_$tag.txt
    done
  done
done
