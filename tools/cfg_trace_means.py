"""Per-kernel means over the timed launches of a traced bench_configs.py run: the JSON lines the
run printed (same process) beside the kernel-trace durations of every launch of each kernel,
the last `steps` launches (the timed loop, after the warm-up) and all of them.
Usage: python tools/cfg_trace_means.py <prof_kernel_trace.csv> <configs.jsonl> [steps]"""
import collections
import csv
import json
import sys

trace, lines = sys.argv[1], sys.argv[2]
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 50
per = collections.OrderedDict()
for r in csv.DictReader(open(trace)):
    name = r["Kernel_Name"]
    if "at::" in name or "rocclr" in name:
        continue
    short = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    per.setdefault(short, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, d in per.items():
    last = d[-steps:]
    print(f"{k:60s} launches {len(d):4d}  mean(all) {sum(d) / len(d):8.2f} us  mean(last {len(last)}) "
          f"{sum(last) / len(last):8.2f} us  min {min(d):8.2f}  max {max(d):8.2f}")
for ln in open(lines):
    if ln.startswith("{"):
        j = json.loads(ln)
        print(f"line: {j['workload'][:70]:70s} ms_per_call {j['ms_per_call']}")
