"""Steady state of the pipelined C2 loop from a rocprofv3 --kernel-trace csv: for the first
`calls` rx_front / rx_back launches (the warm-up plus timed calls; the serial event pass follows),
medians over calls [lo, hi) of each kernel's duration and of its start-to-start period.
Usage: python tools/c2_steady.py <rocprofv3 output dir> <calls> [lo hi]"""
import csv
import glob
import statistics as st
import sys

d, calls = sys.argv[1], int(sys.argv[2])
lo, hi = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (calls // 4, calls - 5)
k = {"F": [], "B": []}
for path in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        n = r.get("Kernel_Name", "")
        key = "F" if "rx_front" in n else "B" if "rx_back" in n else None
        if key:
            k[key].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
for key in k:
    k[key] = sorted(k[key])[:calls]
for key, v in k.items():
    dur = [(e - s) / 1e3 for s, e in v[lo:hi]]
    per = [(v[i + 1][0] - v[i][0]) / 1e3 for i in range(lo, hi - 1)]
    print(f"{key}: duration median {st.median(dur):.2f} us (min {min(dur):.2f}, max {max(dur):.2f}); "
          f"period median {st.median(per):.2f} us, mean {st.mean(per):.2f} us")
# back launches that ran ahead show as short ones: distribution
dur = sorted((e - s) / 1e3 for s, e in k["B"][lo:hi])
print("B durations deciles:", [round(dur[int(q * (len(dur) - 1))], 2) for q in (0, .1, .25, .5, .75, .9, 1)])
