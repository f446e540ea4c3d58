#!/bin/bash
# Round 6 (d): rx_back per-role timing of a skewed launch (UHSDR_TRACE variant) and the mcHF output
# stage inline in the wave pipeline's output role vs the finishing pass (C2 with codec frames).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06d}
V=uhsdr_amd/lib/variants
UHSDR_LIB=$V/libuhsdr_amd_trace.so timeout -k 10 120 python tools/trace_back.py 4096 256 device > gpurun_out/trb_dev_$tag.txt 2>&1 || { tail -20 gpurun_out/trb_dev_$tag.txt; exit 1; }
cat gpurun_out/trb_dev_$tag.txt
UHSDR_LIB=$V/libuhsdr_amd_trace.so timeout -k 10 120 python tools/trace_back.py 4096 256 > gpurun_out/trb_ser_$tag.txt 2>&1 || { tail -20 gpurun_out/trb_ser_$tag.txt; exit 1; }
cat gpurun_out/trb_ser_$tag.txt
for round in 1 2; do
  for v in mcpass mcinline; do
    for board in ovi40 mchf; do
      for steps in 20 1000; do
        UHSDR_LIB=$V/libuhsdr_amd_$v.so timeout -k 10 200 python bench.py --steps $steps --warmup 5 --no-cpu --no-northstar --dst --board $board > gpurun_out/mc_$tag.json 2> gpurun_out/mc_$tag.err || { tail -20 gpurun_out/mc_$tag.err; exit 1; }
        python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], sys.argv[4], d['ms_per_step'], d['value'])" gpurun_out/mc_$tag.json $v $board $steps | tee -a gpurun_out/mc_$tag.txt
      done
    done
  done
done
