#!/bin/bash
# per-role cycles of rx_back for every UHSDR_TRACE variant under uhsdr_amd/lib/variants
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for lib in uhsdr_amd/lib/variants/*.so; do
  echo "== $lib"
  UHSDR_LIB=$lib timeout -k 10 120 python tools/trace_back.py 4096 256 || exit 1
done
