#!/bin/bash
# Round 5: the STREAM schedule (rx_stream) on one GPU box -- a first small parity case under a
# short limit, then its whole test file, the mcHF pipelined / RCCL world-1 tests, and C2 bench
# lines (driver-style 20 steps and 1000 steps) for STREAM against the pipelined split kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-a}
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 240 $T "tests/test_gpu_stream.py::test_stream_paths_match_oracle[48-64]" > gpurun_out/s1_$tag.log 2>&1 || { tail -40 gpurun_out/s1_$tag.log; exit 1; }
tail -3 gpurun_out/s1_$tag.log
timeout -k 10 900 $T tests/test_gpu_stream.py > gpurun_out/stream_$tag.log 2>&1 || { tail -60 gpurun_out/stream_$tag.log; exit 1; }
tail -3 gpurun_out/stream_$tag.log
for s in stream auto; do
  for k in 20 1000; do
    timeout -k 10 300 python bench.py --steps $k --warmup 5 --no-cpu --no-northstar --schedule $s > gpurun_out/b_${s}_${k}_$tag.json 2> gpurun_out/b_${s}_${k}_$tag.err || { tail -20 gpurun_out/b_${s}_${k}_$tag.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d['value'], d['config']['schedule'], d['chain']['kernel_ms'])" gpurun_out/b_${s}_${k}_$tag.json
  done
done
timeout -k 10 600 $T tests/test_gpu_pipelined.py::test_pipelined_mchf_matches_oracle tests/test_gpu_bench_entry.py::test_bench_gather_run_nccl_world1_bit_exact > gpurun_out/misc_$tag.log 2>&1 || { tail -60 gpurun_out/misc_$tag.log; exit 1; }
tail -3 gpurun_out/misc_$tag.log
