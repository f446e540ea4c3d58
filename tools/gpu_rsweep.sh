#!/bin/bash
# front R comparison: R=8 default run (tests + bench) then R=16 bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
bash tools/gpu_quick.sh || exit $?
for r in 16; do
  UHSDR_FRONT_R=$r timeout -k 10 300 python bench.py --steps 500 --warmup 50 --no-cpu > gpurun_out/r${r}_c2.json 2>&1 || exit 1
  UHSDR_FRONT_R=$r timeout -k 10 300 python bench.py --workload northstar --steps 20 --warmup 3 --no-cpu > gpurun_out/r${r}_ns.json 2>&1 || exit 1
  echo "R=$r"; cat gpurun_out/r${r}_c2.json gpurun_out/r${r}_ns.json
done
