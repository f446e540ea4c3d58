#!/bin/bash
# The MFMA FIR's clock in the all-configs process vs a c5fir-only process: GRBM_GUI_ACTIVE per
# dispatch with the kernel trace (one --pmc counter, kernel-trace only), cycles / 8 XCDs / duration.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for run in all:c3,c3spec,c3zoom,c4fm,c4tx,c4txfma,c5,c5fir only:c5fir; do
  name=${run%%:*}; cfgs=${run#*:}
  timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/clk_$name -o clk -- python tools/bench_configs.py --only $cfgs > gpurun_out/clk_$name.jsonl 2> gpurun_out/clk_$name.err || { tail -20 gpurun_out/clk_$name.err; exit 1; }
  grep MFMA gpurun_out/clk_$name.jsonl | cut -c1-60,200-330
done
python - <<'PY'
import csv, glob
for name in ("all", "only"):
    fc = glob.glob(f"gpurun_out/clk_{name}/**/*counter_collection.csv", recursive=True)
    if not fc:
        print(name, "no counter file"); continue
    rows = [r for r in csv.DictReader(open(fc[0])) if "fir_mfma" in r["Kernel_Name"]]
    out = []
    for r in rows:
        cyc = float(r["Counter_Value"]) / 8
        t = None
        for k in ("End_Timestamp", "Stop_Timestamp"):
            if k in r and "Start_Timestamp" in r:
                t = (int(r[k]) - int(r["Start_Timestamp"])) / 1e3
        out.append((cyc, t))
    print(name, "launches", len(out))
    print(" ".join(f"{c/1e3:.0f}kc/{t:.0f}us={c/t/1e3:.2f}GHz" if t else f"{c/1e3:.0f}kc" for c, t in out))
PY
