#!/bin/bash
# Round 6 (b): the skewed wave pipeline (BackSched) -- pipelined / schedule / bench-entry tests, then
# C2 lines at the driver's 20 steps and at 1000 steps (no CPU leg, no north star), and a kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06b}
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_pipelined.py tests/test_gpu_schedules.py tests/test_gpu_bench_entry.py > gpurun_out/t_$tag.log 2>&1 || { tail -80 gpurun_out/t_$tag.log; exit 1; }
tail -3 gpurun_out/t_$tag.log
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-northstar > gpurun_out/b20_${tag}_$i.json 2> gpurun_out/b20_$tag.err || { tail -20 gpurun_out/b20_$tag.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('20', d['ms_per_step'], d['value'], d['chain']['kernel_ms'], d['handoff_timeouts'])" gpurun_out/b20_${tag}_$i.json
timeout -k 10 300 python bench.py --steps 1000 --warmup 50 --no-cpu --no-northstar > gpurun_out/b1k_${tag}_$i.json 2> gpurun_out/b1k_$tag.err || { tail -20 gpurun_out/b1k_$tag.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('1000', d['ms_per_step'], d['value'], d['chain']['kernel_ms'], d['handoff_timeouts'])" gpurun_out/b1k_${tag}_$i.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_$tag -o kt -- python bench.py --steps 20 --warmup 5 --no-cpu --no-northstar > gpurun_out/kt_$tag.log 2>&1 || { tail -20 gpurun_out/kt_$tag.log; exit 1; }
head -4 gpurun_out/kt_$tag/kt_kernel_stats.csv
