#!/bin/bash
# SAM demod A/B: per-role trace (new / old trace builds), C3 line (current / saved library),
# then the whole GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
V=uhsdr_amd/lib/variants
for t in trace; do
  [ -f $V/libuhsdr_amd_$t.so ] || continue
  UHSDR_LIB=$V/libuhsdr_amd_$t.so timeout -k 10 180 python tools/trace_back.py 32768 1024 sam \
      > gpurun_out/sam_$t.txt 2>&1 || { tail -20 gpurun_out/sam_$t.txt; exit 1; }
  tail -4 gpurun_out/sam_$t.txt
done
for lab in cur ${AB:-presam}; do
  lib=uhsdr_amd/lib/libuhsdr_amd.so; [ $lab = cur ] || lib=$V/libuhsdr_amd_$lab.so
  UHSDR_LIB=$lib timeout -k 10 200 python tools/bench_configs.py --only ${ONLY:-c3} > gpurun_out/sam_c3_$lab.jsonl \
      2> gpurun_out/sam_c3_$lab.err || { tail -20 gpurun_out/sam_c3_$lab.err; exit 1; }
  echo "$lab $(cat gpurun_out/sam_c3_$lab.jsonl)"
done
[ -n "$NOTESTS" ] && exit 0
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/sam_tests.log 2>&1 || { tail -30 gpurun_out/sam_tests.log; exit 1; }
tail -3 gpurun_out/sam_tests.log
