#!/bin/bash
# Round 6 (t): per-role trace of the skewed back end with the launch-start marks (wave start offset,
# entry -> skew word consumed), device hand-off.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06t}
for i in 1 2; do
  UHSDR_LIB=uhsdr_amd/lib/traced/libuhsdr_amd_trspec.so timeout -k 10 120 python tools/trace_back.py 4096 256 device > gpurun_out/trb_${tag}_$i.txt 2>&1 || { tail -20 gpurun_out/trb_${tag}_$i.txt; exit 1; }
  cat gpurun_out/trb_${tag}_$i.txt
done
