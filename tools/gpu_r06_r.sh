#!/bin/bash
# Round 6 (r): the pre role's speculative first input of a skewed launch (UHSDR_SPEC_IN) -- per-role
# traces with and without it (device hand-off, the last launch starts skewed), the pipelined tests on
# the variants, then the C2 A/B (20 / 1000 steps).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06r}
T=uhsdr_amd/lib/traced
for v in trnospec trspec; do
  UHSDR_LIB=$T/libuhsdr_amd_$v.so timeout -k 10 120 python tools/trace_back.py 4096 256 device > gpurun_out/trb_${tag}_$v.txt 2>&1 || { tail -20 gpurun_out/trb_${tag}_$v.txt; exit 1; }
  echo "== $v"; cat gpurun_out/trb_${tag}_$v.txt
done
for lib in uhsdr_amd/lib/variants/*.so; do
  UHSDR_LIB=$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pipelined.py -k "long_run or skew_transitions or large_unsync or p48_usb or p48_agc or front_delayed or give_up" > gpurun_out/t_$tag.log 2>&1 || { tail -40 gpurun_out/t_$tag.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/t_$tag.log)"
done
bash tools/gpu_c2_ab.sh $tag
