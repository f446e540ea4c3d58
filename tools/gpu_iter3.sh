#!/bin/bash
# pipelined-mode check: its parity tests, then C2 serial / pipelined
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipelined.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/it3_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/it3_pytest.log
[ $rc -eq 0 ] || { grep -m5 -B5 -A30 "Error\|FAIL" gpurun_out/it3_pytest.log | head -80; exit $rc; }
for m in "--serial" ""; do
  timeout -k 10 200 python bench.py --steps 1000 --warmup 50 --no-cpu --no-northstar $m > gpurun_out/it3_c2$m.json 2> gpurun_out/it3_c2.err || { tail -20 gpurun_out/it3_c2.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['chain']['kernel_ms'])" gpurun_out/it3_c2$m.json "c2$m"
done
