#!/bin/bash
# The configs lines and their kernel trace from ONE process (the rocprof means over
# the same calls as the configs line).  Per-kernel means over the timed launches by
# tools/cfg_trace_means.py; FIR launch durations in order show the clock's drift under load.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-a}
cfgs=${2:-c3,c3spec,c3zoom,c4fm,c4tx,c4txfma,c5,c5fir}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/cfgtrace_$tag -o prof --output-format csv -- python tools/bench_configs.py --only $cfgs > gpurun_out/cfgtrace_$tag.jsonl 2> gpurun_out/cfgtrace_$tag.err || { tail -20 gpurun_out/cfgtrace_$tag.err; exit 1; }
python tools/cfg_trace_means.py gpurun_out/cfgtrace_$tag/prof_kernel_trace.csv gpurun_out/cfgtrace_$tag.jsonl 50
