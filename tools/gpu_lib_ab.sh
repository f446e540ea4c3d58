#!/bin/bash
# A/B of library builds and bench options on one box: each argument is "label|ENV=... |bench args"
# (ENV part may be empty), one north-star line each (WL=c2: the C2 headline line instead).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
tag=$1; shift
for v in "$@"; do
  IFS='|' read label envs bargs <<< "$v"
  out=gpurun_out/${tag}_${label}
  if [ "${WL:-northstar}" = c2 ]; then
    env $envs timeout -k 10 200 python bench.py --steps 1000 --warmup 50 --no-cpu --no-northstar $bargs \
        > $out.json 2> $out.err || { tail -20 $out.err; exit 1; }
  else
    env $envs timeout -k 10 200 python bench.py --workload northstar --steps 100 --warmup 10 --no-cpu $bargs \
        > $out.json 2> $out.err || { tail -20 $out.err; exit 1; }
  fi
  python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['chain']; print(sys.argv[2], d['value'], d['ms_per_step'], c['kernel_ms'], c['hbm_frac'])" $out.json "$label"
done
