#!/bin/bash
# Batched FIR: its parity tests (EXACT bit-exact, MFMA within 1e-5), the C5 FIR lines (EXACT, MFMA)
# and a rocprofv3 kernel trace of both.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-a}
timeout -k 10 300 python -u -m pytest tests/test_gpu_fir.py -x -q --timeout 200 --timeout-method thread > gpurun_out/fir_pytest_$tag.log 2>&1; rc=$?
tail -3 gpurun_out/fir_pytest_$tag.log
[ $rc -eq 0 ] || { tail -60 gpurun_out/fir_pytest_$tag.log; exit $rc; }
timeout -k 10 200 python tools/bench_configs.py --only c5fir --steps 50 > gpurun_out/fir_lines_$tag.jsonl 2>&1 || { tail -20 gpurun_out/fir_lines_$tag.jsonl; exit 1; }
grep '^{' gpurun_out/fir_lines_$tag.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/fir_prof_$tag -o prof --output-format csv -- python tools/bench_configs.py --only c5fir --steps 50 > gpurun_out/fir_prof_$tag.log 2>&1 || { tail -20 gpurun_out/fir_prof_$tag.log; exit 1; }
python tools/kstats.py $(find gpurun_out/fir_prof_$tag -name '*kernel_stats.csv')
if [ "${FIR_PMC:-0}" = 1 ]; then
  PMC_EXTRA="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" bash tools/gpu_pmc_cmd.sh fir_$tag tools/bench_configs.py --only c5fir --steps 10 > gpurun_out/fir_pmc_$tag.json 2> gpurun_out/fir_pmc_$tag.err || { tail -20 gpurun_out/fir_pmc_$tag.err; exit 1; }
  cat gpurun_out/fir_pmc_$tag.json
fi
# A/B against saved builds (uhsdr_amd/lib/variants/*.so), one box
for lib in $(ls uhsdr_amd/lib/variants/*.so 2>/dev/null); do
  v=$(basename $lib .so)
  UHSDR_LIB=$lib timeout -k 10 200 python tools/bench_configs.py --only c5fir --steps 50 > gpurun_out/fir_lines_${tag}_$v.jsonl 2>&1 || { tail -20 gpurun_out/fir_lines_${tag}_$v.jsonl; exit 1; }
  echo "$v:"; grep '^{' gpurun_out/fir_lines_${tag}_$v.jsonl | grep MFMA
  timeout -k 10 200 python tools/bench_configs.py --only c5fir --steps 50 > gpurun_out/fir_lines_${tag}_main2.jsonl 2>&1 || exit 1
  echo "main again:"; grep '^{' gpurun_out/fir_lines_${tag}_main2.jsonl | grep MFMA
done
