#!/bin/bash
# Round 6 (v): the whole GPU suite on the current build (persistent back end the bench default), smoke,
# the driver's bench command and a 1000-step line, the kernel trace of the driver's command, C2 PMC
# passes (device hand-off: a profiler that serialises dispatches cannot run the persistent launch
# beside its fronts), and the other configurations' lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06v}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$tag.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_$tag.log
[ $rc -eq 0 ] || { echo "pytest gpu failed rc=$rc"; tail -60 gpurun_out/pytest_gpu_$tag.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench20_$tag.json 2> gpurun_out/bench20_$tag.err || { tail -30 gpurun_out/bench20_$tag.err; exit 1; }
cat gpurun_out/bench20_$tag.json
timeout -k 10 300 python bench.py --steps 1000 --warmup 5 --no-cpu --no-northstar > gpurun_out/bench1000_$tag.json 2> gpurun_out/bench1000_$tag.err || { tail -30 gpurun_out/bench1000_$tag.err; exit 1; }
cat gpurun_out/bench1000_$tag.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_$tag -o kt -- python bench.py --steps 20 --warmup 5 --no-cpu --no-northstar > gpurun_out/kt_$tag.log 2>&1 || { tail -20 gpurun_out/kt_$tag.log; exit 1; }
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_c2dev_$tag/p$i -o pmc -- python bench.py --no-cpu --no-northstar --steps 20 --warmup 5 --handoff device > gpurun_out/pmc_c2dev_$tag.p$i.log 2>&1 || { echo "device-mode pass $i failed"; tail -5 gpurun_out/pmc_c2dev_$tag.p$i.log; exit 1; }
done
python tools/pmc_summary.py c2dev_$tag > gpurun_out/pmc_c2dev_$tag.json && cat gpurun_out/pmc_c2dev_$tag.json | head -60
timeout -k 10 600 python tools/bench_configs.py > gpurun_out/cfg_$tag.jsonl 2> gpurun_out/cfg_$tag.err || { tail -20 gpurun_out/cfg_$tag.err; exit 1; }
cat gpurun_out/cfg_$tag.jsonl
