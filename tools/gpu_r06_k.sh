#!/bin/bash
# Round 6 (k): tail waves below the roles' issue priority -- per-role trace (mcHF + codec frames) and
# C2 lines, the main build (tails at the roles' priority) against the variant, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06k}
V=uhsdr_amd/lib/variants
UHSDR_LIB=$V/libuhsdr_amd_tr.so timeout -k 10 120 python tools/trace_back.py 4096 256 device dst mchf > gpurun_out/trb_$tag.txt 2>&1 || { tail -20 gpurun_out/trb_$tag.txt; exit 1; }
cat gpurun_out/trb_$tag.txt
for round in 1 2; do
  for lib in uhsdr_amd/lib/libuhsdr_amd.so $V/libuhsdr_amd_prio.so; do
    for opt in "" "--dst" "--dst --board mchf"; do
      for steps in 20 1000; do
        UHSDR_LIB=$lib timeout -k 10 200 python bench.py --steps $steps --warmup 5 --no-cpu --no-northstar $opt > gpurun_out/mc_$tag.json 2> gpurun_out/mc_$tag.err || { tail -20 gpurun_out/mc_$tag.err; exit 1; }
        python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[4], repr(sys.argv[2]), sys.argv[3], d['ms_per_step'], d['value'])" gpurun_out/mc_$tag.json "$opt" $steps $(basename $lib .so) | tee -a gpurun_out/mc_$tag.txt
      done
    done
  done
done
