#!/bin/bash
# Round 6 (u): the persistent back end (uhsdr_rx_set_pipelined 3) -- its tests and the pipelined
# tests on the variant, then C2 lines: the device hand-off (variant "spec") against the persistent
# back end (variant "pers"), 20 / 1000 steps, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06u}
V=uhsdr_amd/lib/variants
UHSDR_LIB=$V/libuhsdr_amd_pers.so timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_persistent.py -k "not p35 and not p4_cw and not p70" > gpurun_out/t_$tag.log 2>&1 || { tail -40 gpurun_out/t_$tag.log; exit 1; }
grep -E "PASS|FAIL|ERROR" gpurun_out/t_$tag.log | tail -20
UHSDR_LIB=$V/libuhsdr_amd_pers.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pipelined.py -k "p48_usb or p48_mchf or p48_agc or long_run or front_delayed or give_up or skew_transitions or large_unsync or mode_switches" > gpurun_out/t2_$tag.log 2>&1 || { tail -40 gpurun_out/t2_$tag.log; exit 1; }
tail -1 gpurun_out/t2_$tag.log
for round in 1 2; do
  for v in "spec device" "pers device" "pers persistent"; do
    set -- $v
    for steps in 20 20 1000; do
      UHSDR_LIB=$V/libuhsdr_amd_$1.so timeout -k 10 200 python bench.py --steps $steps --warmup 5 --no-cpu --no-northstar --handoff $2 > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || { tail -20 gpurun_out/ab_$tag.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], sys.argv[4], d['ms_per_step'], d['value'], d.get('handoff_timeouts'))" gpurun_out/ab_$tag.json $1 $2 $steps | tee -a gpurun_out/ab_$tag.txt
    done
  done
done
