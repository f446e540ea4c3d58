#!/bin/bash
# back-end change check: the RX parity tests (both back ends, every path), role trace, C2 lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paths.py tests/test_gpu_pipelined.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/it2_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/it2_pytest.log
[ $rc -eq 0 ] || { grep -m5 -B5 -A30 "Error\|FAIL" gpurun_out/it2_pytest.log | head -80; exit $rc; }
UHSDR_LIB=uhsdr_amd/lib/variants/libuhsdr_amd_trace.so timeout -k 10 120 python tools/trace_back.py 4096 256 || exit 1
for m in "--serial" ""; do
  timeout -k 10 200 python bench.py --steps 1000 --warmup 50 --no-cpu --no-northstar $m > gpurun_out/it2_c2$m.json 2> gpurun_out/it2_c2.err || { tail -20 gpurun_out/it2_c2.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['chain']['kernel_ms'])" gpurun_out/it2_c2$m.json "c2$m"
done
