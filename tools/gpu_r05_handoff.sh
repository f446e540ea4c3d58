#!/bin/bash
# Round 5: the pipelined mode's device hand-off (uhsdr_rx_set_pipelined 2) -- the pipelined
# parity tests (event and device hand-offs), then C2 lines with each hand-off at the driver's
# 20 steps and at 1000, interleaved on one box, and a kernel timeline of the 20-step device run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-a}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pipelined.py > gpurun_out/ho_test_$tag.log 2>&1 || { tail -60 gpurun_out/ho_test_$tag.log; exit 1; }
tail -1 gpurun_out/ho_test_$tag.log
for rep in 1 2; do
  for k in 20 1000; do
    for ho in event device; do
      f=gpurun_out/ho_${ho}_${k}_${rep}_$tag.json
      timeout -k 10 200 python bench.py --steps $k --warmup 5 --no-cpu --no-northstar --handoff $ho > $f 2> $f.err || { tail -20 $f.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['value'], d['config']['handoff'])" $f
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ho_tl_$tag -o tl --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu --no-northstar --handoff device > gpurun_out/ho_tl_$tag.log 2>&1 || { tail -20 gpurun_out/ho_tl_$tag.log; exit 1; }
python tools/c2_timeline.py gpurun_out/ho_tl_$tag > gpurun_out/ho_tl_$tag.txt && head -60 gpurun_out/ho_tl_$tag.txt
