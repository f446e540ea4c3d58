#!/bin/bash
# Schedule / front-block A/B on the north-star workload (same box, same call): one bench line per
# (schedule, front block, precision) given as "sched:block:prec" arguments.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
tag=$1; shift
for v in "$@"; do
  IFS=: read s fb p <<< "$v"
  out=gpurun_out/${tag}_${s}_${fb}_${p}
  timeout -k 10 200 python bench.py --workload northstar --steps 100 --warmup 10 --no-cpu --schedule $s --front-block $fb --precision $p \
      > $out.json 2> $out.err || { tail -20 $out.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['chain']; print(sys.argv[2], d['value'], d['ms_per_step'], c['kernel_ms'], c['hbm_frac'])" $out.json $v
done
