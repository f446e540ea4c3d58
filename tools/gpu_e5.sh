#!/bin/bash
# Full GPU parity suite on the working tree's library, then a north-star A/B against a
# P48-only build of an earlier revision (uhsdr_amd/lib/variants/libuhsdr_amd_base.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/fma_sweep.py > gpurun_out/fma_sweep.jsonl 2> gpurun_out/fma_sweep.err || { tail -20 gpurun_out/fma_sweep.err; exit 1; }
python - <<'PY'
import json
rows = [json.loads(l) for l in open("gpurun_out/fma_sweep.jsonl")]
ref = [r for r in rows if r.get("refused")]
bad = [r for r in rows if "error" in r or r.get("err", 0) > 1e-5]
print(len(rows), "FMA cases,", len(ref), "refused,", len(bad), "above 1e-5 or failing:", [(r["filter_path"], r["dmod_mode"], r["stereo_enable"], r.get("err", r.get("error"))) for r in bad])
print("max err of the rest:", max(r["err"] for r in rows if r not in bad and r not in ref))
PY
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 120 --timeout-method thread > gpurun_out/e5_pytest.log 2>&1 || { tail -60 gpurun_out/e5_pytest.log; exit 1; }
tail -3 gpurun_out/e5_pytest.log
V=uhsdr_amd/lib/variants
bash tools/gpu_lib_ab.sh e5 "base|UHSDR_LIB=$V/libuhsdr_amd_base.so|--schedule fused" "new||--schedule fused" "basefma|UHSDR_LIB=$V/libuhsdr_amd_base.so|--schedule fused --precision fma" "newfma||--schedule fused --precision fma" "base2|UHSDR_LIB=$V/libuhsdr_amd_base.so|--schedule fused" "new2||--schedule fused" "newchain||--schedule chain"
