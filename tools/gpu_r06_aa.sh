#!/bin/bash
# Round 6 (aa): the persistent back end's host-memory reads moved to a control tail wave (variant "ctl")
# against the committed build's instance ("pers"): persistent tests, per-call timing, C2 20 x3 / 1000.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06z}
V=uhsdr_amd/lib/variants
UHSDR_LIB=$V/libuhsdr_amd_ctl.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_persistent.py -k "not p35 and not p4_cw and not p70" > gpurun_out/t_$tag.log 2>&1 || { tail -40 gpurun_out/t_$tag.log; exit 1; }
tail -1 gpurun_out/t_$tag.log
UHSDR_LIB=$V/libuhsdr_amd_ctlpdbg.so timeout -k 10 60 python tools/debug_persist3.py 60 5 | tail -22 || exit 1
for round in 1 2; do
  for v in pers ctl; do
    for steps in 20 20 20 1000; do
      UHSDR_LIB=$V/libuhsdr_amd_$v.so timeout -k 10 200 python bench.py --steps $steps --warmup 5 --no-cpu --no-northstar > gpurun_out/z_$tag.json 2> gpurun_out/z_$tag.err || { tail -20 gpurun_out/z_$tag.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['ms_per_step'], d['value'], d['handoff_timeouts'])" gpurun_out/z_$tag.json $v $steps | tee -a gpurun_out/z_$tag.txt
    done
  done
done
