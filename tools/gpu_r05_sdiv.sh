#!/bin/bash
# Round 5: atanf's reduction quotient by reciprocal + one correction (UHSDR_ATAN_SHORTDIV variant):
# the exhaustive device check, the SAM / FM / AM parity tests on the variant, then C3 SAM and C4 FM
# lines against the main build, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
V=uhsdr_amd/lib/variants/libuhsdr_amd_sdiv.so
timeout -k 10 120 ./tools/micro/atan_div_check | tee gpurun_out/atan_div_check.txt
UHSDR_LIB=$V timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "sam or SAM or fm or FM or am_ or libm or p70 or p1_" > gpurun_out/sdiv_test.log 2>&1 || { tail -40 gpurun_out/sdiv_test.log; exit 1; }
tail -1 gpurun_out/sdiv_test.log
for rep in 1 2; do
  for v in main sdiv; do
    if [ $v = sdiv ]; then L=$V; else L=uhsdr_amd/lib/libuhsdr_amd.so; fi
    UHSDR_LIB=$L timeout -k 10 200 python tools/bench_configs.py --only c3,c4fm > gpurun_out/sdiv_${v}_$rep.jsonl 2>&1 || { tail -20 gpurun_out/sdiv_${v}_$rep.jsonl; exit 1; }
    python -c "import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'): d=json.loads(l); print(sys.argv[2], d['workload'][:20], d['ms_per_call'], d['hbm_frac'], d.get('kernel_ms'))" gpurun_out/sdiv_${v}_$rep.jsonl $v
  done
done
