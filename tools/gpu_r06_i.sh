#!/bin/bash
# Round 6 (i): the wave pipeline's tail waves (the board's output stage and the stores off the
# output role) -- per-role traces with codec frames (OVI40, mcHF), the pipelined / schedule / mcHF /
# bench-entry tests, and C2 lines for OVI40, OVI40 + codec frames and mcHF + codec frames.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06i}
V=uhsdr_amd/lib/variants
for run in "device" "device dst" "device dst mchf"; do
  echo "== $run"
  UHSDR_LIB=$V/libuhsdr_amd_tr.so timeout -k 10 120 python tools/trace_back.py 4096 256 $run > gpurun_out/trb_$tag.txt 2>&1 || { tail -20 gpurun_out/trb_$tag.txt; exit 1; }
  cat gpurun_out/trb_$tag.txt
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pipelined.py tests/test_gpu_schedules.py tests/test_gpu_bench_entry.py tests/test_gpu_parity.py tests/test_gpu_paths.py > gpurun_out/t_$tag.log 2>&1 || { tail -40 gpurun_out/t_$tag.log; exit 1; }
tail -2 gpurun_out/t_$tag.log
for round in 1 2; do
  for opt in "" "--dst" "--dst --board mchf" "--board mchf"; do
    for steps in 20 1000; do
      timeout -k 10 200 python bench.py --steps $steps --warmup 5 --no-cpu --no-northstar $opt > gpurun_out/mc_$tag.json 2> gpurun_out/mc_$tag.err || { tail -20 gpurun_out/mc_$tag.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(repr(sys.argv[2]), sys.argv[3], d['ms_per_step'], d['value'])" gpurun_out/mc_$tag.json "$opt" $steps | tee -a gpurun_out/mc_$tag.txt
    done
  done
done
