#!/usr/bin/env python3
"""Hardware-queue isolation of a pipeline rank's streams, measured on one MI355X.

Two stream layouts, each with the streams a PP rank creates (compute, send, recv, head, capture),
PyTorch's stream pool initialised, and 2 RCCL-internal pool streams per communicator of the
busiest rank (the last stage at PP=8: 1 stage pair + 7 head pairs = 16 streams):

  round2     compute on the null stream, send / recv / head / capture from torch's stream pool
             (what round 2 shipped)
  dedicated  runtime/streams.py RankStreams: every role on a full-CU-mask stream

For each waiting role (send, recv, head) a kernel spins on it (as an RCCL receive waits for its
peer) with barrier packets queued behind it on the 16 RCCL-style streams; every other role must
still complete its work within 1.5 s (compute replays a captured decode-like graph).
Writes ``--out`` (JSON).  ``--log-only`` just creates the dedicated streams (run it under
AMD_LOG_LEVEL=4 to see HIP's hardware-queue assignment)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/queue_probe.json")
    ap.add_argument("--log-only", action="store_true")
    ap.add_argument("--copies-only", action="store_true",
                    help="only the host->device copy coupling check (run with and without "
                         "HSA_ENABLE_SDMA=0)")
    a = ap.parse_args()
    import torch
    from distributed_llm_inference import ops
    from distributed_llm_inference.runtime.streams import RankStreams, isolation_matrix
    C = ops.native()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if a.log_only:
        print("=== creating dedicated RankStreams", file=sys.stderr, flush=True)
        rs = RankStreams(dev, "dedicated")
        print("=== creating 4 pool streams", file=sys.stderr, flush=True)
        ps = [C.stream_create(0, 0, 0) for _ in range(4)]
        print("=== done", rs.describe(), file=sys.stderr, flush=True)
        for p in ps:
            C.stream_destroy(p)
        rs.close()
        return

    if a.copies_only:
        rs = RankStreams(dev, "dedicated")
        res = {"HSA_ENABLE_SDMA": os.environ.get("HSA_ENABLE_SDMA", "<unset: SDMA on>")}
        for kind, ck in (("memcpy", False), ("copy_kernel", True)):
            m = isolation_matrix(rs.streams, ("send", "recv", "head"), dev, host_copies=True,
                                 copy_kernels=ck)
            res[kind] = {"isolated": all(v for row in m.values() for v in row.values()),
                         "matrix": m}
        print(json.dumps(res), flush=True)
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
        rs.close()
        return
    x = torch.randn(2048, 2048, device=dev, dtype=torch.bfloat16)
    w = torch.randn(2048, 2048, device=dev, dtype=torch.bfloat16)
    out = {"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES", "<unset: HIP default 4>"),
           "hip_priority_range": None, "layouts": {}}
    internal = [torch.cuda.ExternalStream(C.stream_create(0, 0, 0), device=dev) for _ in range(16)]
    torch.cuda.Stream()   # PyTorch's pool exists in every real rank (graph capture uses it)

    def graph_on(cap):
        g = torch.cuda.CUDAGraph()
        cap.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cap):
            for _ in range(2):
                y = x @ w
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=cap):
            y = x
            for _ in range(8):
                y = torch.nn.functional.silu(y @ w)
        torch.cuda.synchronize()
        return g

    layouts = {}
    r2 = {"compute": torch.cuda.default_stream(dev), "send": torch.cuda.Stream(dev),
          "recv": torch.cuda.Stream(dev), "head": torch.cuda.Stream(dev),
          "capture": torch.cuda.Stream(dev)}
    layouts["round2"] = r2
    rs = RankStreams(dev, "dedicated")
    ded = dict(rs.streams)
    ded["null"] = torch.cuda.default_stream(dev)   # observer: is a CU-mask stream "blocking"?
    layouts["dedicated"] = ded
    for name, streams in layouts.items():
        g = graph_on(streams["capture"])
        res = {}
        for bar in (False, True):
            m = isolation_matrix(streams, ("send", "recv", "head"), dev,
                                 barrier_streams=internal if bar else (), graph=g)
            res["with_rccl_barriers" if bar else "spin_only"] = m
        ok = all(v for mode in res.values() for row in mode.values()
                 for k, v in row.items() if k != "null")
        out["layouts"][name] = {"isolated": ok, "matrix": res}
        print(name, "isolated" if ok else "SHARED", json.dumps(res), flush=True)
    out["dedicated_describe"] = rs.describe()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    for s in internal:
        C.stream_destroy(s.cuda_stream)
    rs.close()


if __name__ == "__main__":
    main()
