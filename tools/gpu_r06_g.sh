#!/bin/bash
# Round 6 (g): per-role timing of skewed rx_back launches with int32 codec frames, OVI40 and mcHF
# (the mcHF stage inline in the output role vs the finishing pass).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06g}
V=uhsdr_amd/lib/variants
for run in "tr_pass device dst" "tr_pass device dst mchf" "tr_inl device dst mchf"; do
  set -- $run; v=$1; shift
  echo "== $v $*"
  UHSDR_LIB=$V/libuhsdr_amd_$v.so timeout -k 10 120 python tools/trace_back.py 4096 256 "$@" > gpurun_out/trb_$tag.txt 2>&1 || { tail -20 gpurun_out/trb_$tag.txt; exit 1; }
  cat gpurun_out/trb_$tag.txt
done
