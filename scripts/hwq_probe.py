#!/usr/bin/env python3
"""How many hardware queues with a spinning (peer-waiting) kernel can one GPU hold before a queue
with ready work stops being scheduled?

One process creates ``n`` dedicated (CU-masked: one HSA hardware queue each) streams, parks a
spinning wait kernel (runtime/streams.py's receive wait, bounded by a deadline) on ``n - 1`` of
them, then launches a trivial kernel on the last one and records whether it completes within
``--window`` seconds while the spinners still spin.  The GPU's scheduler maps a limited number of
user queues at a time; when more queues hold work than that, the others wait to be mapped - and a
queue parked on a spinning wave never becomes idle, so it may never give its slot up.  Eight
pipeline ranks sharing ONE GPU (the DLI_SHARE_GPU rehearsal) each bring their dedicated streams
plus HIP's pool queues; one rank per GPU (production) brings ~9.  Writes ``--out`` (JSON)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--counts", default="8,16,24,28,32,36,40,48,64")
    ap.add_argument("--window", type=float, default=2.0)
    ap.add_argument("--spin-timeout", type=float, default=8.0)
    ap.add_argument("--out", default="gpurun_out/hwq_probe.json")
    a = ap.parse_args()
    import torch
    from distributed_llm_inference import ops
    C = ops.native()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    out = torch.zeros(1, dtype=torch.int32, device=dev)
    res = []
    for n in (int(v) for v in a.counts.split(",")):
        handles = [C.stream_create(0, 1, 0) for _ in range(n)]
        flags = C.HostWords(2)
        flags.set(0, 0)
        flags.set(1, 0)
        for h in handles[:-1]:
            C.wait_geq(flags.dev_ptr(0), 1, a.spin_timeout, flags.dev_ptr(1), 1, h, 0)
        time.sleep(0.2)   # let every spinner start
        last = torch.cuda.ExternalStream(handles[-1], device=dev)
        C.touch(out, handles[-1])
        ev = torch.cuda.Event()
        ev.record(last)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < a.window and not ev.query():
            time.sleep(1e-3)
        done = bool(ev.query())
        lat = time.perf_counter() - t0
        flags.set(0, 1)
        torch.cuda.synchronize(dev)
        expired = flags.get(1) != 0
        for h in handles:
            C.stream_destroy(h)
        r = {"queues": n, "spinning": n - 1, "ready_queue_ran": done,
             "latency_s": round(lat, 4), "spinner_deadline_hit": expired}
        print(json.dumps(r), flush=True)
        res.append(r)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump({"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES", "<unset>"),
                   "results": res}, f, indent=1)


if __name__ == "__main__":
    main()
