#!/bin/bash
# Round 6 (h): the output role's coalesced (LDS-staged) stores -- per-role traces with codec frames
# (OVI40, mcHF inline, mcHF finishing pass), mcHF parity on the inline variant, then C2 lines for
# OVI40 / OVI40+dst / mcHF+dst per variant (interleaved, two rounds).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06h}
V=uhsdr_amd/lib/variants
for run in "tr_pass device dst" "tr_inl device dst mchf" "tr_pass device dst mchf"; do
  set -- $run; v=$1; shift
  echo "== $v $*"
  UHSDR_LIB=$V/libuhsdr_amd_$v.so timeout -k 10 120 python tools/trace_back.py 4096 256 "$@" > gpurun_out/trb_$tag.txt 2>&1 || { tail -20 gpurun_out/trb_$tag.txt; exit 1; }
  cat gpurun_out/trb_$tag.txt
done
UHSDR_LIB=$V/libuhsdr_amd_inl.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pipelined.py -k "mchf or handoff" > gpurun_out/t_$tag.log 2>&1 || { tail -40 gpurun_out/t_$tag.log; exit 1; }
tail -2 gpurun_out/t_$tag.log
for round in 1 2; do
  for v in pass inl; do
    for opt in "" "--dst" "--dst --board mchf"; do
      for steps in 20 1000; do
        UHSDR_LIB=$V/libuhsdr_amd_$v.so timeout -k 10 200 python bench.py --steps $steps --warmup 5 --no-cpu --no-northstar $opt > gpurun_out/mc_$tag.json 2> gpurun_out/mc_$tag.err || { tail -20 gpurun_out/mc_$tag.err; exit 1; }
        python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], repr(sys.argv[3]), sys.argv[4], d['ms_per_step'], d['value'])" gpurun_out/mc_$tag.json $v "$opt" $steps | tee -a gpurun_out/mc_$tag.txt
      done
    done
  done
done
