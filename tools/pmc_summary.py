#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (gpurun_out/pmc_<tag>/p*/pmc_counter_collection.csv) per kernel:
mean counter value per dispatch for the rx_front / rx_back kernels, plus derived metrics.
FETCH_SIZE / WRITE_SIZE are in KB; on gfx950 FETCH_SIZE counts half the bytes of wide
coalesced streaming reads (MI355X_MICROARCH.md §HBM), so HBM read bytes = 2 x FETCH_SIZE KB."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

tag = sys.argv[1]
base = os.path.join("gpurun_out", f"pmc_{tag}")
vals = defaultdict(lambda: defaultdict(list))
meta = {}
for f in sorted(glob.glob(os.path.join(base, "p*", "pmc_counter_collection.csv"))):
    for row in csv.DictReader(open(f)):
        name = row["Kernel_Name"]
        for k in ("rx_front", "rx_back_dec", "rx_back_out", "rx_back", "rx_fm", "rx_notch", "tx_voice", "tx_iq", "spectrum_frames",
                  "spectrum_accumulate", "spectrum_zoom", "fir_batch_direct", "fir_batch", "fir_mfma"):
            if k in name:
                break
        else:
            continue
        key = (row["Dispatch_Id"], f)
        vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
        meta[k] = dict(grid=int(row["Grid_Size"]), wg=int(row["Workgroup_Size"]), lds=int(row["LDS_Block_Size"]),
                       vgpr=int(row["VGPR_Count"]), sgpr=int(row["SGPR_Count"]), scratch=int(row["Scratch_Size"]),
                       kernel=name)
out = {}
for k, cs in vals.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    d = dict(meta[k])
    d.update({c: round(v, 1) for c, v in m.items()})
    if "FETCH_SIZE" in m:
        d["hbm_read_bytes_corrected"] = 2 * m["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in m:
        d["hbm_write_bytes"] = m["WRITE_SIZE"] * 1024
    if "SQ_INSTS_VALU" in m and "SQ_WAVES" in m:
        d["valu_per_wave"] = round(m["SQ_INSTS_VALU"] / m["SQ_WAVES"], 1)
        d["lds_per_wave"] = round(m.get("SQ_INSTS_LDS", 0) / m["SQ_WAVES"], 1)
    if "SQ_ACTIVE_INST_VALU" in m and "SQ_WAVE_CYCLES" in m:
        d["valu_active_frac_of_wave_cycles"] = round(m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVE_CYCLES"], 3)
    if "SQ_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
        d["busy_frac"] = round(m["SQ_BUSY_CYCLES"] / max(m["GRBM_GUI_ACTIVE"], 1), 3)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
        # MFMA busy cycles summed over the chip's 1024 SIMDs; GRBM_GUI_ACTIVE summed over its 8 XCDs
        d["mfma_busy_frac"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / max(m["GRBM_GUI_ACTIVE"] / 8 * 1024, 1), 3)
    out[k] = d
# the bench line of every pass (p<i>.log): which mode the counters come from, and that no pass ran
# a stalled or failed chain (the device hand-off's give-up is an error since round 6, but an event-mode
# run is the one that cannot stall under the profiler's serialised dispatch)
runs = []
for f in sorted(glob.glob(os.path.join(base, "p*.log"))):
    for line in open(f):
        if line.startswith("{") and '"metric"' in line:
            b = json.loads(line)
            cfg = b.get("config", {})
            runs.append({"pass": os.path.basename(f)[:-4], "ms_per_step": b.get("ms_per_step"),
                         "pipelined": cfg.get("pipelined"), "handoff": cfg.get("handoff"),
                         "schedule": cfg.get("schedule"), "handoff_timeouts": b.get("handoff_timeouts")})
if runs:
    out["_runs"] = runs
print(json.dumps(out, indent=1))
