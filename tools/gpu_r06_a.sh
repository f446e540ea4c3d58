#!/bin/bash
# Round 6 (a): the device hand-off's failure contract and the STREAM removal on the GPU -- the
# pipelined / schedule / bench-entry tests (forced give-up, delayed fronts), smoke, the driver's
# 20-step bench line, its kernel trace, and the C2 PMC passes in event mode (cannot stall under
# the profiler's serialised dispatch).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06a}
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_pipelined.py tests/test_gpu_schedules.py tests/test_gpu_bench_entry.py > gpurun_out/t_$tag.log 2>&1 || { tail -80 gpurun_out/t_$tag.log; exit 1; }
tail -3 gpurun_out/t_$tag.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/b20_$tag.json 2> gpurun_out/b20_$tag.err || { tail -20 gpurun_out/b20_$tag.err; exit 1; }
cat gpurun_out/b20_$tag.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_$tag -o kt -- python bench.py --steps 20 --warmup 5 --no-cpu --no-northstar > gpurun_out/kt_$tag.log 2>&1 || { tail -20 gpurun_out/kt_$tag.log; exit 1; }
bash tools/gpu_pmc.sh c2_$tag --steps 20 --warmup 5 --handoff event || exit 1
python tools/pmc_summary.py c2_$tag > gpurun_out/pmc_c2_$tag.json && cat gpurun_out/pmc_c2_$tag.json
