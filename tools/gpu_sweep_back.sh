#!/bin/bash
# rx_back pipelined vs fused across batch sizes (64-frame calls), then the per-config benches.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/sweep_back.txt
: > $out
for C in 16384 65536 131072 262144 1048576; do
  for F in 0 1; do
    UHSDR_BACK_FUSED=$F timeout -k 10 120 python bench.py --no-cpu --no-northstar --channels $C --frames 64 --steps 50 --warmup 5 > gpurun_out/sw.json 2>gpurun_out/sw.err || { tail -5 gpurun_out/sw.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/sw.json'));print($C, $F, d['value'], d['chain']['kernel_ms'])" | tee -a $out
  done
done
timeout -k 10 300 python tools/bench_configs.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err || { tail -20 gpurun_out/configs.err; exit 1; }
cat gpurun_out/configs.jsonl
