"""Kernel timeline of a rocprofv3 --kernel-trace run (csv): for the rx_ kernels, in start order,
each kernel's duration and the gap since the previous rx_ kernel ended (negative = overlap).
Usage: python tools/c2_timeline.py <rocprofv3 output dir>"""
import csv
import glob
import sys

rows = []
for path in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        n = r.get("Kernel_Name", r.get("KernelName", ""))
        if "rx_" in n:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n.split("<")[0].split("(")[0]))
rows.sort()
print(f"{len(rows)} rx kernels")
# the last 20 calls' worth of kernels (the timed region plus the event pass follow the warm-up)
prev_end = None
t0 = rows[0][0] if rows else 0
for s, e, n in rows[-160:]:
    gap = "" if prev_end is None else f"{(s - prev_end) / 1e3:8.2f}"
    print(f"{(s - t0) / 1e3:10.2f} us  {n[:28]:28s} dur {(e - s) / 1e3:7.2f} us  gap {gap}")
    prev_end = e if prev_end is None else max(prev_end, e)
