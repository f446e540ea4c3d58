#!/bin/bash
# Round 5: same-box A/B of the back-end pipeline forms on C2 (pipelined split kernels, 20 and 1000
# steps, two interleaved rounds): lockstep (one barrier per call, libuhsdr_amd_lock.so) against the
# progress-word pipeline at 1 and 2 units per call (u1, u2).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
tag=${1:-a}
for rep in 1 2; do
  for lib in lock u1 u2; do
    for k in 20 1000; do
      f=gpurun_out/ab_${lib}_${k}_${rep}_$tag.json
      UHSDR_LIB=uhsdr_amd/lib/variants/libuhsdr_amd_$lib.so timeout -k 10 300 python bench.py --steps $k --warmup 5 --no-cpu --no-northstar > $f 2> $f.err || { tail -20 $f.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d['chain']['kernel_ms'])" $f
    done
  done
done
