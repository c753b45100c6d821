#!/usr/bin/env python3
"""Multi-process variant of scripts/hwq_probe.py: do P processes sharing ONE GPU, each parking
spinning wait kernels on some of its dedicated streams (as pipeline ranks do on send / recv /
head), still get a kernel on another of their streams scheduled?

Each child creates ``--streams`` dedicated streams, waits at a common barrier, parks a spinning
wait (deadline ``--spin-timeout``) on ``--spinners`` of them, then launches a trivial kernel on
the last stream and records whether it completes within ``--window`` s while every process's
spinners still spin.  The GPU scheduler maps queues of a limited number of processes (and
queues) at a time; a process whose queues are not mapped makes no progress until another
process's queues drain - and queues parked on spinning waves never drain on their own.
Writes ``--out`` (JSON): per process count, how many processes' ready kernels ran."""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child(rank, a, barrier, q):
    import torch
    from distributed_llm_inference import ops
    C = ops.native()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    out = torch.zeros(1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    handles = [C.stream_create(0, 1, 0) for _ in range(a.streams)]
    flags = C.HostWords(2)
    flags.set(0, 0)
    flags.set(1, 0)
    barrier.wait()
    for h in handles[:a.spinners]:
        C.wait_geq(flags.dev_ptr(0), 1, a.spin_timeout, flags.dev_ptr(1), 1, h, 0)
    barrier.wait()
    time.sleep(0.3)
    last = torch.cuda.ExternalStream(handles[-1], device=dev)
    C.touch(out, handles[-1])
    ev = torch.cuda.Event()
    ev.record(last)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < a.window and not ev.query():
        time.sleep(1e-3)
    ran = bool(ev.query())
    lat = time.perf_counter() - t0
    barrier.wait()          # every process measured while all spinners still spin
    flags.set(0, 1)
    torch.cuda.synchronize(dev)
    for h in handles:
        C.stream_destroy(h)
    q.put({"rank": rank, "ran": ran, "latency_s": round(lat, 4),
           "spinner_deadline_hit": flags.get(1) != 0})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", default="2,4,8")
    ap.add_argument("--streams", type=int, default=5)
    ap.add_argument("--spinners", type=int, default=3)
    ap.add_argument("--window", type=float, default=3.0)
    ap.add_argument("--spin-timeout", type=float, default=10.0)
    ap.add_argument("--out", default="gpurun_out/hwq_probe_mp.json")
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    res = []
    for P in (int(v) for v in a.procs.split(",")):
        barrier = ctx.Barrier(P)
        q = ctx.Queue()
        ps = [ctx.Process(target=child, args=(r, a, barrier, q)) for r in range(P)]
        for p in ps:
            p.start()
        rows = []
        for _ in range(P):
            rows.append(q.get(timeout=300))
        for p in ps:
            p.join(60)
        r = {"procs": P, "streams_per_proc": a.streams, "spinners_per_proc": a.spinners,
             "ready_kernels_ran": sum(x["ran"] for x in rows),
             "max_latency_s": max(x["latency_s"] for x in rows),
             "deadline_hits": sum(x["spinner_deadline_hit"] for x in rows)}
        print(json.dumps(r), flush=True)
        res.append(r)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
