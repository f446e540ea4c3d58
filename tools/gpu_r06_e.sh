#!/bin/bash
# Round 6 (e): per-role timing of a skewed rx_back launch (UHSDR_TRACE variant), then the C2 A/B
# of the main build against the variants, and the skewed pipeline's parity tests on the variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06e}
V=uhsdr_amd/lib/variants
UHSDR_LIB=$V/libuhsdr_amd_trace.so timeout -k 10 120 python tools/trace_back.py 4096 256 device > gpurun_out/trb_dev_$tag.txt 2>&1 || { tail -20 gpurun_out/trb_dev_$tag.txt; exit 1; }
cat gpurun_out/trb_dev_$tag.txt
UHSDR_LIB=$V/libuhsdr_amd_r6new.so timeout -k 10 300 python tools/debug_skew.py || exit 1
bash tools/gpu_c2_ab.sh $tag
