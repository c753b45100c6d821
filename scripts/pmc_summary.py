"""Per-kernel averages of every counter in rocprofv3 --pmc CSV runs (counter_collection.csv),
plus mean duration, for the kernels of scripts/pmc_decode_kernels.py."""
import collections
import csv
import glob
import os
import re
import sys

vals = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for root in sys.argv[1:]:
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        seen = set()
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
            name = re.sub(r"\(.*", "", name).replace("void ", "")[:60]
            if not name.startswith("dli::"):
                continue
            vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
            key = (r["Dispatch_Id"], root)
            if key not in seen:
                seen.add(key)
                dur[name].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k in sorted(vals):
    d = sorted(dur[k])
    print(f"== {k}  dispatches={len(d)}  median duration {d[len(d)//2]/1e3:.1f} us (under PMC)")
    for c in sorted(vals[k]):
        v = vals[k][c]
        print(f"   {c:<32} {sum(v)/len(v):>18.1f}")
    a = {c: sum(v) / len(v) for c, v in vals[k].items()}
    if "SQ_WAVE_CYCLES" in a and a["SQ_WAVE_CYCLES"]:
        w = a["SQ_WAVE_CYCLES"]
        print(f"   -> wave time: waiting {100*a.get('SQ_WAIT_ANY',0)/w:.1f} %, issue-stalled "
              f"{100*a.get('SQ_WAIT_INST_ANY',0)/w:.1f} %, issuing {100*a.get('SQ_ACTIVE_INST_ANY',0)/w:.1f} %")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in a and a.get("GRBM_GUI_ACTIVE"):
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs: per-XCD cycles = GUI / 8; 256 CUs x 4 SIMDs
        cyc = a["GRBM_GUI_ACTIVE"] / 8
        us = d[len(d) // 2] / 1e3
        print(f"   -> clock {cyc / (us * 1e-6) / 1e9:.2f} GHz, MFMA util "
              f"{100 * a['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * 1024):.1f} %")
    if "FETCH_SIZE" in a:
        print(f"   -> FETCH_SIZE {a['FETCH_SIZE']/1e3:.1f} MB per dispatch")
