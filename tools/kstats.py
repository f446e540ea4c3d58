"""Print the rx_/tx_/spectrum_/fir_ kernels of a rocprofv3 --stats kernel summary (mean us)."""
import csv
import sys

for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        n = r["Name"]
        if any(k in n for k in ("rx_", "tx_", "spectrum", "fir_", "cfft")):
            print(f"{float(r['AverageNs']) / 1e3:10.2f} us  x{r['Calls']:>5}  {n[:90]}")
