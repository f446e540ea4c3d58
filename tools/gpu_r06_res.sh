#!/bin/bash
# Round 6 (res): mode 3 with and without the back end's CU reservation (variant "nores":
# UHSDR_BACK_RESERVE=0) against the same sources' variant "base", C2 20 x3 / 1000, two rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06res}
V=uhsdr_amd/lib/variants
for round in 1 2; do
  for v in base nores; do
    for steps in 20 20 20 1000; do
      UHSDR_LIB=$V/libuhsdr_amd_$v.so timeout -k 10 200 python bench.py --steps $steps --warmup 5 --no-cpu --no-northstar > gpurun_out/res_$tag.json 2> gpurun_out/res_$tag.err || { tail -20 gpurun_out/res_$tag.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['ms_per_step'], d['value'], d['handoff_timeouts'])" gpurun_out/res_$tag.json $v $steps | tee -a gpurun_out/res_$tag.txt
    done
  done
done
