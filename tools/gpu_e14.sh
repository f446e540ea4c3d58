#!/bin/bash
# TX pipelined mode: its parity tests and the TX suite, then the config lines serial vs pipelined
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tx_pipelined.py tests/test_gpu_tx.py tests/test_gpu_pipelined.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/e14_pytest.log 2>&1 || { tail -60 gpurun_out/e14_pytest.log; exit 1; }
tail -1 gpurun_out/e14_pytest.log
for m in serial pipe; do
  flag=""; [ $m = serial ] && flag="--serial"
  timeout -k 10 400 python tools/bench_configs.py --only c4tx,c4fm $flag > gpurun_out/e14_cfg_$m.jsonl 2> gpurun_out/e14_cfg_$m.err || { tail -20 gpurun_out/e14_cfg_$m.err; exit 1; }
  python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(sys.argv[2], d['workload'][:40], d['ms_per_call'], d.get('kernel_ms'), d['hbm_frac'], d['finite'])" gpurun_out/e14_cfg_$m.jsonl $m
done
