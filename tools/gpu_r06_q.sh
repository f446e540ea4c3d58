#!/bin/bash
# Round 6 (q): tail-wave count of the demodulator-free back end (UHSDR_BACK_TAILS 4 / 2 / 1, with
# the second-chance peek): the pipelined tests on each variant, then the C2 A/B (20 / 1000 steps).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06q}
for lib in uhsdr_amd/lib/variants/*.so; do
  UHSDR_LIB=$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pipelined.py -k "long_run or skew_transitions or large_unsync or p48_usb or p48_agc" > gpurun_out/t_$tag.log 2>&1 || { tail -40 gpurun_out/t_$tag.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/t_$tag.log)"
done
bash tools/gpu_c2_ab.sh $tag
