#!/bin/bash
# Round 5: rx_stream timelines (UHSDR_STREAM_TRACE variants: lazy / eager publish), then the STREAM
# parity tests and C2 lines of the main build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-a}
for v in ${VARIANTS:-strace}; do
  UHSDR_LIB=uhsdr_amd/lib/variants/libuhsdr_amd_$v.so timeout -k 10 120 python tools/trace_stream.py > gpurun_out/trace_${v}_$tag.txt 2>&1 || { tail -20 gpurun_out/trace_${v}_$tag.txt; exit 1; }
  cat gpurun_out/trace_${v}_$tag.txt
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_stream.py > gpurun_out/stream_$tag.log 2>&1 || { tail -60 gpurun_out/stream_$tag.log; exit 1; }
tail -2 gpurun_out/stream_$tag.log
for k in 20 1000; do
  timeout -k 10 300 python bench.py --steps $k --warmup 5 --no-cpu --no-northstar --schedule stream > gpurun_out/b_stream_${k}_$tag.json 2> gpurun_out/b_stream_${k}_$tag.err || { tail -20 gpurun_out/b_stream_${k}_$tag.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d['value'], d['config']['schedule'], d['chain']['kernel_ms'])" gpurun_out/b_stream_${k}_$tag.json
done
if [ -n "$HOSTCOST" ]; then
  timeout -k 10 200 python tools/host_cost.py > gpurun_out/host_cost_$tag.txt 2>&1 || { tail -20 gpurun_out/host_cost_$tag.txt; exit 1; }
  cat gpurun_out/host_cost_$tag.txt
fi
