#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_spectrum.py -x -q > gpurun_out/pytest_spec.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_spec.log
[ $rc -eq 0 ] || exit $rc
for o in avg both; do timeout -k 10 120 python tools/bench_spectrum.py --outputs $o || exit 1; done
timeout -k 10 120 python tools/bench_spectrum.py --fft 512 || exit 1
timeout -k 10 120 python tools/bench_spectrum.py --fft 256 || exit 1
timeout -k 10 120 python tools/bench_spectrum.py --auto 1 || exit 1
