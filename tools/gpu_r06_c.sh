#!/bin/bash
# Round 6 (c): steady-state timelines (rocprofv3 kernel trace, 300 pipelined C2 calls) of the main
# build and the variants, plus 20 / 1000-step lines per build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06c}
libs="uhsdr_amd/lib/libuhsdr_amd.so $(ls uhsdr_amd/lib/variants/*.so 2>/dev/null)"
for lib in $libs; do
  v=$(basename $lib .so)
  UHSDR_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ss_${tag}_$v -o ss --output-format csv -- python bench.py --steps 300 --warmup 5 --no-cpu --no-northstar > gpurun_out/ss_${tag}_$v.log 2>&1 || { tail -20 gpurun_out/ss_${tag}_$v.log; exit 1; }
  echo "== $v"; python tools/c2_steady.py gpurun_out/ss_${tag}_$v 305 | tee gpurun_out/ss_${tag}_$v.txt
done
bash tools/gpu_c2_ab.sh $tag
