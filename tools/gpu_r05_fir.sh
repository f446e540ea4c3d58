#!/bin/bash
# Round 5: the MFMA FIR with the taps' B fragments held in registers (fir_mfma_rb, 8 waves per
# workgroup, one LDS read per four MFMAs) against round 4's fir_mfma (both operands from LDS; the
# norb variant library).  FIR parity tests, the c5fir configs line for each (alternated twice), a
# waves sweep, and the rocprofv3 kernel-trace summary over the same calls as the configs line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-a}
NORB=uhsdr_amd/lib/variants/libuhsdr_amd_norb.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fir.py > gpurun_out/f1_$tag.log 2>&1 || { tail -60 gpurun_out/f1_$tag.log; exit 1; }
tail -1 gpurun_out/f1_$tag.log
for rep in 1 2; do
  timeout -k 10 300 python tools/bench_configs.py --only c5fir --steps 50 > gpurun_out/fir_rb_${rep}_$tag.jsonl 2> gpurun_out/fir_rb_${rep}_$tag.err || { tail -20 gpurun_out/fir_rb_${rep}_$tag.err; exit 1; }
  UHSDR_LIB=$NORB timeout -k 10 300 python tools/bench_configs.py --only c5fir --steps 50 > gpurun_out/fir_norb_${rep}_$tag.jsonl 2> gpurun_out/fir_norb_${rep}_$tag.err || { tail -20 gpurun_out/fir_norb_${rep}_$tag.err; exit 1; }
  for v in rb norb; do
    python -c "import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(sys.argv[2], d['workload'][-40:], d['waves_per_workgroup'], d['ms_per_call'], d['alg_tflops'])" gpurun_out/fir_${v}_${rep}_$tag.jsonl $v
  done
done
for w in 4 6; do
  timeout -k 10 300 python tools/bench_configs.py --only c5fir --steps 50 --fir-waves $w > gpurun_out/fir_rb_w${w}_$tag.jsonl 2>&1 || { tail -20 gpurun_out/fir_rb_w${w}_$tag.jsonl; exit 1; }
  grep MFMA gpurun_out/fir_rb_w${w}_$tag.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fir_$tag -o fir -- python tools/bench_configs.py --only c5fir --steps 50 > gpurun_out/prof_fir_$tag.log 2>&1 || { tail -30 gpurun_out/prof_fir_$tag.log; exit 1; }
cat gpurun_out/prof_fir_$tag.log
f=$(ls gpurun_out/prof_fir_$tag/*/fir_kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && cat "$f"
exit 0
