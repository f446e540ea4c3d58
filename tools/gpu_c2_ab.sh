#!/bin/bash
# C2 A/B of library builds (uhsdr_amd/lib/variants/*.so and the main build), interleaved on one
# box: the driver-style 20-step line twice and a 1000-step line per build, per round.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-ab}
libs="uhsdr_amd/lib/libuhsdr_amd.so $(ls uhsdr_amd/lib/variants/*.so 2>/dev/null)"
for round in 1 2; do
  for lib in $libs; do
    v=$(basename $lib .so)
    for steps in 20 20 1000; do
      UHSDR_LIB=$lib timeout -k 10 200 python bench.py --steps $steps --warmup 5 --no-cpu --no-northstar > gpurun_out/c2ab_${tag}.json 2> gpurun_out/c2ab_${tag}.err || { tail -20 gpurun_out/c2ab_${tag}.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['ms_per_step'], d['value'], d['chain']['kernel_ms'])" gpurun_out/c2ab_${tag}.json $v $steps | tee -a gpurun_out/c2ab_${tag}.txt
    done
  done
done
