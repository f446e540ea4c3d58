#!/bin/bash
# rx_chain iteration: parity of every path under every schedule, the 1M-channel sampled check,
# then north-star lines per schedule and precision (kernel times from the bench's events).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-chain}
timeout -k 10 900 python -u -m pytest tests/test_gpu_paths.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${tag}_pytest.log 2>&1 || { tail -60 gpurun_out/${tag}_pytest.log; exit 1; }
tail -3 gpurun_out/${tag}_pytest.log
for s in chain fused; do
  for p in exact fma; do
    timeout -k 10 200 python bench.py --workload northstar --steps 100 --warmup 10 --no-cpu --schedule $s --precision $p \
        > gpurun_out/${tag}_ns_${s}_${p}.json 2> gpurun_out/${tag}_ns_${s}_${p}.err || { tail -20 gpurun_out/${tag}_ns_${s}_${p}.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['chain']; print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], c['kernel_ms'], c['hbm_frac'])" gpurun_out/${tag}_ns_${s}_${p}.json $s $p
  done
done
