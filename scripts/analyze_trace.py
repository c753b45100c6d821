#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (CSV or rocpd .db) for the decode phase of bench.py.

Decode steps are delimited by the sampling kernel (one per micro-batch step); the last
``--steps`` decode steps are aggregated per kernel (short names), with per-step time, share,
achieved bandwidth for GEMMs (given the shape table) and the gaps between kernels.
"""
import argparse
import collections
import csv
import re


def short(name: str) -> str:
    if name.startswith("Cijk") or name.startswith("Custom_Cijk"):
        m = re.search(r"MT(\d+x\d+x\d+)", name)
        return f"hipBLASLt_GEMM[{m.group(1) if m else '?'}]" + ("_SK" if "_SK" in name else "")
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "")
    return name[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=4, help="decode micro-batch steps to aggregate")
    ap.add_argument("--marker", default="sample_kernel")
    ap.add_argument("--cycle", default="", help="KERNEL:N - per-position means of KERNEL's calls "
                    "(~TEXT:N: every kernel whose name contains TEXT)")
    a = ap.parse_args()
    if a.trace.endswith(".db"):  # rocprofv3 rocpd (SQLite) output
        import sqlite3
        con = sqlite3.connect(a.trace)
        rows = [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e}
                for n, s, e in con.execute("select name, start, end from kernels")]
    else:
        rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(marks) < a.steps + 1:
        raise SystemExit(f"only {len(marks)} marker kernels")
    lo, hi = marks[-a.steps - 1] + 1, marks[-1] + 1
    seg = rows[lo:hi]
    t0 = int(seg[0]["Start_Timestamp"])
    t1 = int(seg[-1]["End_Timestamp"])
    busy = collections.Counter()
    calls = collections.Counter()
    for r in seg:
        k = short(r["Kernel_Name"])
        busy[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        calls[k] += 1
    total_busy = sum(busy.values())
    wall = t1 - t0
    print(f"decode window: {a.steps} micro-batch steps, wall {wall/1e6:.3f} ms "
          f"({wall/1e6/a.steps:.3f} ms/step), kernel busy {total_busy/1e6:.3f} ms "
          f"({100*total_busy/wall:.1f}% of wall), kernels {len(seg)}")
    # idle time between consecutive kernels (end of one -> start of the next; overlaps count 0)
    gaps = []
    end = int(seg[0]["End_Timestamp"])
    for r in seg[1:]:
        s = int(r["Start_Timestamp"])
        gaps.append(max(0, s - end))
        end = max(end, int(r["End_Timestamp"]))
    if gaps:
        gs = sorted(gaps)
        print(f"inter-kernel gaps: {sum(gaps)/1e3/a.steps:.1f} us/step over {len(gaps)/a.steps:.0f} gaps/step, "
              f"median {gs[len(gs)//2]/1e3:.2f} us, p90 {gs[int(len(gs)*0.9)]/1e3:.2f} us, "
              f"max {gs[-1]/1e3:.1f} us")
    print(f"{'kernel':<60} {'calls/step':>10} {'us/step':>10} {'share':>7}")
    for k, v in busy.most_common():
        print(f"{k:<60} {calls[k]/a.steps:>10.1f} {v/1e3/a.steps:>10.1f} {100*v/total_busy:>6.1f}%")
    # per-position split of a kernel that serves several projections of a layer (the split-K tile
    # GEMM runs QKV, O and down in that order): mean duration of the i-th call in each cycle
    if a.cycle:
        name, n = a.cycle.rsplit(":", 1)
        n = int(n)
        pos = [[] for _ in range(n)]
        step_bounds = marks[-a.steps - 1:]
        for s0, s1 in zip(step_bounds[:-1], step_bounds[1:]):   # cycles restart every step
            durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                    for r in rows[s0 + 1:s1 + 1]
                    if (name[1:] in short(r["Kernel_Name"]) if name.startswith("~")
                        else short(r["Kernel_Name"]) == name)]
            for j, d in enumerate(durs[:len(durs) - len(durs) % n]):
                pos[j % n].append(d)
        print(f"\n{name}: mean us per position in cycles of {n} (per step, {len(pos[0])} cycles)")
        for i in range(n):
            d = pos[i]
            if d:
                print(f"  position {i}: {sum(d) / len(d) / 1e3:8.1f} us  (min {min(d) / 1e3:.1f})")


if __name__ == "__main__":
    main()
