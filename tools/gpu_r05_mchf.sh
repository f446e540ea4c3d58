#!/bin/bash
# Round 5: the mcHF output stage -- inline in the back ends' line_out4 (fused, FM, chain), a
# finishing pass after the wave pipeline (rx_back, rx_stream).  mcHF parity tests, then lines for
# mcHF and OVI40 at the C2 shape (wave pipeline) and at 1M x 64 (fused back end), each with its HBM
# traffic (FETCH_SIZE / WRITE_SIZE passes over a short serial run).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-a}
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_parity.py -k mchf > gpurun_out/m1_$tag.log 2>&1 || { tail -60 gpurun_out/m1_$tag.log; exit 1; }
tail -1 gpurun_out/m1_$tag.log
timeout -k 10 900 $T tests/test_gpu_pipelined.py tests/test_gpu_stream.py tests/test_gpu_i2s.py > gpurun_out/m2_$tag.log 2>&1 || { tail -60 gpurun_out/m2_$tag.log; exit 1; }
tail -1 gpurun_out/m2_$tag.log
for w in c2 northstar; do
  for b in mchf ovi40; do
    f=gpurun_out/bm_${w}_${b}_$tag.json
    if [ $w = c2 ]; then K=1000; else K=50; fi
    timeout -k 10 300 python bench.py --workload $w --steps $K --warmup 5 --no-cpu --no-northstar --board $b --dst > $f 2> $f.err || { tail -20 $f.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d['value'], d['chain']['kernel_ms'], d['config'].get('board'))" $f
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_m_${w}_${b}_$tag/$c -o pmc -- python bench.py --workload $w --steps 10 --warmup 3 --no-cpu --no-northstar --serial --board $b --dst > gpurun_out/pmc_m_${w}_${b}_$tag.$c.log 2>&1 || { tail -20 gpurun_out/pmc_m_${w}_${b}_$tag.$c.log; exit 1; }
    done
  done
done
python - "$tag" <<'PY'
import csv, glob, collections, sys
tag = sys.argv[1]
for w in ("c2", "northstar"):
    for b in ("mchf", "ovi40"):
        acc = collections.defaultdict(list)
        for f in glob.glob(f"gpurun_out/pmc_m_{w}_{b}_{tag}/*/pmc_counter_collection.csv"):
            for r in csv.DictReader(open(f)):
                if "rx_" in r["Kernel_Name"]:
                    acc[(r["Kernel_Name"].split("<")[0].split("(")[0].replace("void ", ""), r["Counter_Name"])].append(float(r["Counter_Value"]))
        for k, v in sorted(acc.items()):
            print(w, b, k[0], k[1], round(sum(v) / len(v)), "KB per launch")
PY
