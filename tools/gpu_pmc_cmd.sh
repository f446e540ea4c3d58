#!/bin/bash
# PMC counter passes over an arbitrary python command (kernel-trace only, no sys/runtime trace).
# Usage: [PMC_EXTRA="COUNTERS..."] tools/gpu_pmc_cmd.sh <tag> <script.py> [args...]
# (PMC_EXTRA: one more pass, e.g. "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE")
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/pmc_$tag
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" ${PMC_EXTRA:+"$PMC_EXTRA"}; do
  i=$((i+1))
  echo "=== pass $i: $grp" >&2
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_$tag/p$i -o pmc -- python "$@" > gpurun_out/pmc_$tag/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 gpurun_out/pmc_$tag/p$i.log; exit 1; }
done
python tools/pmc_summary.py $tag
echo PMC_DONE >&2
