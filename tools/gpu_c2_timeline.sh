#!/bin/bash
# C2 timeline on one GPU box: host submission cost per call (tools/host_cost.py), then a
# rocprofv3 kernel trace of the driver-style 20-step bench (no CPU / north-star legs) whose
# per-kernel start / end times tools/c2_timeline.py turns into gaps and overlaps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-a}
timeout -k 10 200 python tools/host_cost.py > gpurun_out/host_cost_$tag.txt 2>&1 || { tail -20 gpurun_out/host_cost_$tag.txt; exit 1; }
cat gpurun_out/host_cost_$tag.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl_$tag -o tl --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu --no-northstar > gpurun_out/tl_$tag.log 2>&1 || { tail -20 gpurun_out/tl_$tag.log; exit 1; }
python tools/c2_timeline.py gpurun_out/tl_$tag > gpurun_out/tl_$tag.txt && cat gpurun_out/tl_$tag.txt
