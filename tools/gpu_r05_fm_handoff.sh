#!/bin/bash
# Round 5: the device hand-off for rx_fm (FM-RX, C4): pipelined parity tests, then the C4 FM line
# with the event and the device hand-off, interleaved on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-a}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pipelined.py tests/test_gpu_parity.py -k "fm or FM or device_handoff" > gpurun_out/fmho_test_$tag.log 2>&1 || { tail -60 gpurun_out/fmho_test_$tag.log; exit 1; }
tail -1 gpurun_out/fmho_test_$tag.log
for rep in 1 2; do
  for ho in event device; do
    timeout -k 10 200 python tools/bench_configs.py --only c4fm --handoff $ho > gpurun_out/fmho_${ho}_${rep}_$tag.jsonl 2>&1 || { tail -20 gpurun_out/fmho_${ho}_${rep}_$tag.jsonl; exit 1; }
    python -c "import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'): d=json.loads(l); print(sys.argv[2], d['ms_per_call'], d['msamples_per_s'], d['hbm_frac'], d.get('kernel_ms'))" gpurun_out/fmho_${ho}_${rep}_$tag.jsonl $ho
  done
done
