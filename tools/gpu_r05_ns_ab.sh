#!/bin/bash
# Round 5: north-star A/B of compile variants (P48-only builds), EXACT and FMA, interleaved twice:
#   bash tools/gpu_r05_ns_ab.sh <tag> <variant> ...   (uhsdr_amd/lib/variants/libuhsdr_amd_<variant>.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
tag=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    for p in exact fma; do
      f=gpurun_out/ns_${v}_${p}_${rep}_$tag.json
      UHSDR_LIB=uhsdr_amd/lib/variants/libuhsdr_amd_$v.so timeout -k 10 300 python bench.py --workload northstar --steps 100 --warmup 10 --no-cpu --precision $p > $f 2> $f.err || { tail -20 $f.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].split('/')[-1], d['ms_per_step'], round(d['chain']['hbm_frac'],4), d['chain']['kernel_ms'])" $f
    done
  done
done
