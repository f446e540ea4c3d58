#!/bin/bash
# C4 SSB-TX in the serial mode (EXACT, FMA): the line and a rocprofv3 kernel trace, so tx_voice2
# and tx_iq are timed alone (the pipelined lines overlap them).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-a}
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/txs_prof_$tag -o prof --output-format csv -- python tools/bench_configs.py --serial --only c4tx,c4txfma --steps 50 > gpurun_out/txs_prof_$tag.log 2>&1 || { tail -20 gpurun_out/txs_prof_$tag.log; exit 1; }
grep '^{' gpurun_out/txs_prof_$tag.log
python tools/kstats.py $(find gpurun_out/txs_prof_$tag -name '*kernel_stats.csv')
