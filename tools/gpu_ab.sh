#!/bin/bash
# A/B of compile variants (uhsdr_amd/lib/variants/*.so, `make variant`) and env settings on the
# north-star and C2 workloads: kernel times of each build.
# Usage: tools/gpu_ab.sh <tag> ["ENV=v ..." ...]   (each extra argument: one env setting to try
# with the main build)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
tag=${1:-ab}; shift
run() {  # run <label> <env...>
  local v=$1; shift
  for wl in northstar c2; do
    steps=20; [ $wl = c2 ] && steps=500
    env "$@" timeout -k 10 200 python bench.py --workload $wl --steps $steps --warmup 3 --no-cpu --no-northstar > gpurun_out/ab_${tag}_${v}_${wl}.json 2> gpurun_out/ab_${tag}_${v}_${wl}.err || { tail -20 gpurun_out/ab_${tag}_${v}_${wl}.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d.get('chain',{}).get('kernel_ms', d.get('kernel_ms')))" gpurun_out/ab_${tag}_${v}_${wl}.json $v $wl
  done
}
for lib in uhsdr_amd/lib/libuhsdr_amd.so uhsdr_amd/lib/variants/*.so; do
  [ -f "$lib" ] || continue
  run $(basename $lib .so) UHSDR_LIB=$lib
done
i=0
for e in "$@"; do i=$((i+1)); run env$i $e; done
