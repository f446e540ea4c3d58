#!/bin/bash
# Round 6 (ab3): the control wave also reads the next call's data on a launch's first call (variant "first")
# against the committed build (variant "head"): persistent tests, then C2 20 x3 / 1000, interleaved.

set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06ab3}
V=uhsdr_amd/lib/variants
UHSDR_LIB=$V/libuhsdr_amd_first.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_persistent.py -k "not p35 and not p4_cw and not p70" > gpurun_out/t_$tag.log 2>&1 || { tail -40 gpurun_out/t_$tag.log; exit 1; }
tail -1 gpurun_out/t_$tag.log
for round in 1 2; do
  for lib in $V/libuhsdr_amd_head.so $V/libuhsdr_amd_first.so; do
    for steps in 20 20 20 1000; do
      UHSDR_LIB=$lib timeout -k 10 200 python bench.py --steps $steps --warmup 5 --no-cpu --no-northstar > gpurun_out/ab2_$tag.json 2> gpurun_out/ab2_$tag.err || { tail -20 gpurun_out/ab2_$tag.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['ms_per_step'], d['value'], d['handoff_timeouts'])" gpurun_out/ab2_$tag.json $(basename $lib .so) $steps | tee -a gpurun_out/ab2_$tag.txt
    done
  done
done
