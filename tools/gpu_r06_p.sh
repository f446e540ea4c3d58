#!/bin/bash
# Round 6 (p): the pre role's second-chance peek (UHSDR_LATE_EXT) for running ahead:
# the pipelined tests on the variant, then the C2 A/B against the main build (20 / 1000 steps).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06p}
UHSDR_LIB=uhsdr_amd/lib/variants/libuhsdr_amd_late.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pipelined.py -k "long_run or front_delayed or skew_transitions or large_unsync or give_up or mode_switches or toggle or p48_usb or p48_mchf or p48_agc" > gpurun_out/t_$tag.log 2>&1 || { tail -40 gpurun_out/t_$tag.log; exit 1; }
tail -2 gpurun_out/t_$tag.log
UHSDR_LIB=uhsdr_amd/lib/variants/libuhsdr_amd_late.so timeout -k 10 300 python tools/debug_skew.py || exit 1
bash tools/gpu_c2_ab.sh $tag
