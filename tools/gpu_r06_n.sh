#!/bin/bash
# Round 6 (n): the MFMA FIR in a process of its own at the default warm-up and
# after a longer one, with its kernel trace; then C2 PMC passes in the bench's own device hand-off
# mode (no signal kernel any more, so a serialised dispatch order should no longer stall it).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06n}
for w in 5 200; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fir_${tag}_w$w -o fir -- python tools/bench_configs.py --only c5fir --warmup $w --steps 100 > gpurun_out/fir_${tag}_w$w.jsonl 2> gpurun_out/fir_${tag}_w$w.err || { tail -20 gpurun_out/fir_${tag}_w$w.err; exit 1; }
  cat gpurun_out/fir_${tag}_w$w.jsonl
  grep -i "fir_mfma" gpurun_out/fir_${tag}_w$w/fir_kernel_stats.csv | cut -c1-200
done
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_c2dev_$tag/p$i -o pmc -- python bench.py --no-cpu --no-northstar --steps 20 --warmup 5 > gpurun_out/pmc_c2dev_$tag/p$i.log 2>&1 || { echo "device-mode pass $i failed"; tail -5 gpurun_out/pmc_c2dev_$tag/p$i.log; exit 0; }
done
python tools/pmc_summary.py c2dev_$tag > gpurun_out/pmc_c2dev_$tag.json && cat gpurun_out/pmc_c2dev_$tag.json
