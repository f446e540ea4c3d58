#!/bin/bash
# The whole -m gpu suite on the current build, then a same-box A/B of the north-star line against
# a saved library (uhsdr_amd/lib/variants/libuhsdr_amd_<base>.so), EXACT and FMA, interleaved.
# Usage: tools/gpu_ab_run.sh <tag> <base>
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
tag=$1; base=$2
B=UHSDR_LIB=uhsdr_amd/lib/variants/libuhsdr_amd_${base}.so
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { tail -60 gpurun_out/pytest_gpu.log; exit $rc; }
bash tools/gpu_lib_ab.sh $tag "$base|$B|" "new||" "${base}fma|$B|--precision fma" "newfma||--precision fma" "${base}2|$B|" "new2||"
