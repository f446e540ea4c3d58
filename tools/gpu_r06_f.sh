#!/bin/bash
# Round 6 (f): the whole GPU suite on the current build, smoke, the driver's bench command, and the
# C2 kernel trace of the driver's command.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06f}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$tag.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_$tag.log
[ $rc -eq 0 ] || { echo "pytest gpu failed rc=$rc"; tail -60 gpurun_out/pytest_gpu_$tag.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench20_$tag.json 2> gpurun_out/bench20_$tag.err || { tail -30 gpurun_out/bench20_$tag.err; exit 1; }
cat gpurun_out/bench20_$tag.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_$tag -o kt -- python bench.py --steps 20 --warmup 5 --no-cpu --no-northstar > gpurun_out/kt_$tag.log 2>&1 || { tail -20 gpurun_out/kt_$tag.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ss_$tag -o ss -- python bench.py --steps 300 --warmup 5 --no-cpu --no-northstar > gpurun_out/ss_$tag.log 2>&1 || { tail -20 gpurun_out/ss_$tag.log; exit 1; }
python tools/c2_steady.py gpurun_out/ss_$tag 305 | tee gpurun_out/ss_$tag.txt
timeout -k 10 600 python tools/bench_configs.py --only c3,c3spec,c4fm,c4tx,c4txfma,c5,c5fir > gpurun_out/cfg_$tag.jsonl 2> gpurun_out/cfg_$tag.err || { tail -20 gpurun_out/cfg_$tag.err; exit 1; }
cat gpurun_out/cfg_$tag.jsonl
