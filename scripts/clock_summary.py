"""Per-kernel effective clock from a rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace CSV run:
sum(GRBM_GUI_ACTIVE) / sum(duration) over the last dispatches of each kernel name."""
import collections
import csv
import glob
import os
import re
import sys

root = sys.argv[1]
cc = glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)
if not cc:
    raise SystemExit(f"no counter_collection.csv under {root}")
rows = list(csv.DictReader(open(cc[0])))
print("columns:", list(rows[0].keys()))
cyc = collections.defaultdict(float)
dur = collections.defaultdict(float)
n = collections.Counter()
for r in rows:
    if r.get("Counter_Name") != "GRBM_GUI_ACTIVE":
        continue
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name).replace("void ", "")[:70]
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) if "End_Timestamp" in r else 0
    cyc[name] += float(r["Counter_Value"])
    dur[name] += d
    n[name] += 1
print("(GRBM_GUI_ACTIVE is summed over the 8 XCDs: divide by 8 for the per-XCD clock)")
for k in sorted(dur, key=lambda k: -dur[k])[:16]:
    mhz = cyc[k] / dur[k] * 1e3 if dur[k] else float("nan")
    print(f"{k:<70} n={n[k]:>6} busy {dur[k]/1e6:9.2f} ms  GUI_ACTIVE/ns -> {mhz:7.0f} MHz")
