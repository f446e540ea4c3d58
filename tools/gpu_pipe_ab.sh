#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_lib_ab.sh pab "ser||" "pipe||--pipelined" "serfma||--precision fma" "pipefma||--precision fma --pipelined" "ser2||" "pipe2||--pipelined" || exit 1
timeout -k 10 300 python tools/bench_configs.py --only c3,c3pipe > gpurun_out/pab_c3.jsonl 2> gpurun_out/pab_c3.err || { tail gpurun_out/pab_c3.err; exit 1; }
cat gpurun_out/pab_c3.jsonl
