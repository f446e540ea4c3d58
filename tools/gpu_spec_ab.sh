#!/bin/bash
# A/B of the spectrum kernels' waves per workgroup (UHSDR_SPEC_WAVES builds under uhsdr_amd/lib/variants)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for lib in uhsdr_amd/lib/libuhsdr_amd.so uhsdr_amd/lib/variants/libuhsdr_amd_sw2.so uhsdr_amd/lib/variants/libuhsdr_amd_sw1.so; do
  v=$(basename $lib .so)
  UHSDR_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_spectrum.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/spec_ab_pytest_$v.log 2>&1 || { tail -30 gpurun_out/spec_ab_pytest_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/spec_ab_pytest_$v.log)"
  UHSDR_LIB=$lib timeout -k 10 200 python tools/bench_configs.py --only c3spec > gpurun_out/spec_ab_$v.jsonl 2> gpurun_out/spec_ab_$v.err || { tail -20 gpurun_out/spec_ab_$v.err; exit 1; }
  cut -c1-260 gpurun_out/spec_ab_$v.jsonl
done
