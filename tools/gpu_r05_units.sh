#!/bin/bash
# Round 5: the non-lockstep unit pipeline of rx_back / rx_stream -- parity tests of every kernel
# that runs the pipeline roles, then C2 lines (pipelined split kernels and STREAM, 20 and 1000
# steps) of the main build and of the BACK_UNITS = 1 / 4 variants, the C3 SAM line, a stream trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-a}
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 240 $T "tests/test_gpu_pipelined.py::test_pipelined_matches_oracle[pipe-p48_usb]" > gpurun_out/u0_$tag.log 2>&1 || { tail -40 gpurun_out/u0_$tag.log; exit 1; }
tail -1 gpurun_out/u0_$tag.log
timeout -k 10 900 $T tests/test_gpu_pipelined.py tests/test_gpu_stream.py tests/test_gpu_schedules.py tests/test_gpu_cw.py > gpurun_out/u1_$tag.log 2>&1 || { tail -60 gpurun_out/u1_$tag.log; exit 1; }
tail -1 gpurun_out/u1_$tag.log
line() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d['value'], d['config']['schedule'], d['chain']['kernel_ms'])" $1; }
for lib in main u1 u4; do
  if [ $lib = main ]; then L=""; else L=uhsdr_amd/lib/variants/libuhsdr_amd_$lib.so; fi
  for s in auto stream; do
    for k in 20 1000; do
      f=gpurun_out/bu_${lib}_${s}_${k}_$tag.json
      UHSDR_LIB=$L timeout -k 10 300 python bench.py --steps $k --warmup 5 --no-cpu --no-northstar --schedule $s > $f 2> $f.err || { tail -20 $f.err; exit 1; }
      line $f
    done
  done
done
timeout -k 10 300 python tools/bench_configs.py --only c3 > gpurun_out/c3_$tag.jsonl 2> gpurun_out/c3_$tag.err || { tail -20 gpurun_out/c3_$tag.err; exit 1; }
cat gpurun_out/c3_$tag.jsonl
UHSDR_LIB=uhsdr_amd/lib/variants/libuhsdr_amd_strace.so timeout -k 10 120 python tools/trace_stream.py > gpurun_out/trace_u_$tag.txt 2>&1 || { tail -20 gpurun_out/trace_u_$tag.txt; exit 1; }
cat gpurun_out/trace_u_$tag.txt
