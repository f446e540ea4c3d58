#!/bin/bash
# The whole -m gpu suite on the current build, then per-config lines (bench_configs.py) of a saved
# library (uhsdr_amd/lib/variants/libuhsdr_amd_<base>.so) and of the current build, interleaved.
# Usage: tools/gpu_cfg_ab.sh <tag> <base> <configs> [bench_configs args]
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
tag=$1; base=$2; only=$3; shift 3
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { tail -60 gpurun_out/pytest_gpu.log; exit $rc; }
for round in 1 2; do
  for v in $base new; do
    if [ $v = new ]; then envs=""; else envs="UHSDR_LIB=uhsdr_amd/lib/variants/libuhsdr_amd_${base}.so"; fi
    env $envs timeout -k 10 300 python tools/bench_configs.py --only $only "$@" > gpurun_out/${tag}_${v}${round}.jsonl 2> gpurun_out/${tag}_${v}${round}.err || { tail -20 gpurun_out/${tag}_${v}${round}.err; exit 1; }
    python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(sys.argv[2], d.get('workload','')[:40], d.get('ms_per_call'), d.get('kernel_ms'), d.get('hbm_frac'), d.get('finite'))" gpurun_out/${tag}_${v}${round}.jsonl $v$round
  done
done
