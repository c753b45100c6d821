"""Top kernels of a rocprofv3 --stats kernel_stats.csv: name (short), calls, total ms, share."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
tot = sum(float(r["TotalDurationNs"]) for r in rows)
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
print(f"total GPU kernel time {tot / 1e6:.1f} ms over {len(rows)} kernels")
for r in rows[:n]:
    name = re.sub(r"\(.*", "", r["Name"].replace("(anonymous namespace)::", "")).replace("void ", "")
    if name.startswith(("Cijk", "Custom_Cijk")):
        m = re.search(r"MT(\d+x\d+x\d+)", name)
        name = "hipBLASLt_GEMM[" + (m.group(1) if m else "?") + "]"
    t = float(r["TotalDurationNs"])
    print(f"{t / 1e6:10.1f} ms {100 * t / tot:5.1f} %  {int(r['Calls']):6d} calls  {name[:90]}")
