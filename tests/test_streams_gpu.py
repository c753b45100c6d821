"""Hardware-queue isolation of a pipeline rank's streams (runtime/streams.py) on the MI355X.

Round-2 verdict item 1(a): with the box's default 4 hardware queues per process, a kernel that
waits on another rank (RCCL / IPC receive, a send whose peer has not posted, the rotating head's
receive) must never sit in the same in-order hardware queue as the stage's compute or the other
transfers.  Every stream a rank creates is built in ``init_pipeline_rank`` order (RankStreams,
PyTorch's pool, RCCL-style internal streams); a kernel then spins on each waiting role in turn,
with RCCL-style barrier packets queued behind it on 16 pool streams, and a real decode-graph
replay on ``compute`` plus copies on every other role must complete while it spins.
"""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _small_stage_graph(dev, capture):
    """A decode-like graph (GEMMs + the framework's RMSNorm kernel) captured on ``capture``."""
    from distributed_llm_inference import ops
    x = torch.randn(256, 1024, device=dev, dtype=torch.bfloat16)
    w = torch.randn(1024, 1024, device=dev, dtype=torch.bfloat16) * 0.03
    nw = torch.ones(1024, device=dev, dtype=torch.bfloat16)
    cur = torch.cuda.current_stream()
    capture.wait_stream(cur)
    with torch.cuda.stream(capture):
        y = ops.rms_norm(x @ w, nw, 1e-5)[0]
    cur.wait_stream(capture)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=capture):
        y = x
        for _ in range(6):
            y = ops.rms_norm(y @ w, nw, 1e-5)[0]
    torch.cuda.synchronize()
    return g


def test_dedicated_streams_have_their_own_hardware_queues(gpu):
    from distributed_llm_inference import ops
    from distributed_llm_inference.runtime.streams import (WAITING_ROLES, RankStreams,
                                                           isolation_matrix)
    assert os.environ.get("GPU_MAX_HW_QUEUES", "4") == "4", "test the box default"
    C = ops.native()
    dev = torch.device("cuda", 0)
    rs = RankStreams(dev, "dedicated")
    torch.cuda.Stream()   # PyTorch's stream pool, as in every real rank (graph capture)
    internal = [torch.cuda.ExternalStream(C.stream_create(0, 0, 0), device=dev) for _ in range(16)]
    try:
        ncu = torch.cuda.get_device_properties(dev).multi_processor_count
        assert all(v == ncu for v in rs.describe()["cu_per_stream"].values())
        g = _small_stage_graph(dev, rs.capture)
        m = isolation_matrix(rs.streams, WAITING_ROLES, dev, barrier_streams=internal, graph=g)
        stuck = {w: [o for o, ok in row.items() if not ok] for w, row in m.items()}
        assert not any(stuck.values()), f"roles stalled behind a waiting kernel: {stuck}"
    finally:
        for s in internal:
            C.stream_destroy(s.cuda_stream)
        rs.close()


def test_runtime_host_copies_are_not_coupled_across_streams(gpu):
    """Host <-> device copies the runtime makes per step (staging uploads, token returns) are
    copy KERNELS on the issuing stream reading / writing device-mapped host memory: one queued on
    a stream behind a spinning receive (the rotating head's uploads) must not hold up another
    stream's copies (a hipMemcpyAsync goes through a copy queue the process's streams share:
    scripts/queue_probe.py --copies-only, profiles/streams/copies_*.json)."""
    from distributed_llm_inference.runtime.streams import (WAITING_ROLES, RankStreams,
                                                           isolation_matrix)
    dev = torch.device("cuda", 0)
    rs = RankStreams(dev, "dedicated")
    try:
        m = isolation_matrix(rs.streams, WAITING_ROLES, dev, host_copies=True, copy_kernels=True)
        stuck = {w: [o for o, ok in row.items() if not ok] for w, row in m.items()}
        assert not any(stuck.values()), f"copies stalled behind a waiting stream's copy: {stuck}"
    finally:
        rs.close()


def test_staging_and_token_ring_roundtrip(gpu):
    """The executor's host-mapped staging (one copy kernel per step) and the token ring deliver
    exactly the bytes written, slot after slot."""
    from distributed_llm_inference.runtime.executor import _Staging
    from distributed_llm_inference.runtime.streams import HostTokenRing
    dev = torch.device("cuda", 0)
    st = _Staging(64, 16, 4, dev)
    for it in range(9):
        st.acquire()
        st.h["positions"][:7] = torch.arange(7, dtype=torch.int32) + it
        st.h["seq_lens"][:3] = torch.tensor([it, 2 * it, 3], dtype=torch.int32)
        st.h["block_tables"][:2] = it
        st.upload("positions", 7)
        st.upload("seq_lens", 3)
        st.upload("block_tables", 2)
        st.release()
        torch.cuda.synchronize()
        assert torch.equal(st.d["positions"][:7].cpu(), torch.arange(7, dtype=torch.int32) + it)
        assert st.d["seq_lens"][:3].tolist() == [it, 2 * it, 3]
        assert (st.d["block_tables"][:2] == it).all()
    ring = HostTokenRing(dev, 512, slots=4)
    outs = []
    for it in range(10):
        tok = torch.arange(300, device=dev, dtype=torch.int32) * (it + 1)
        outs.append((it, *ring.take(tok)))
        if len(outs) > 2:   # consume two behind, as the pipeline does
            j, host, ev = outs.pop(0)
            ev.synchronize()
            assert host.tolist() == (torch.arange(300, dtype=torch.int32) * (j + 1)).tolist()
    # more unconsumed takes than slots: the ring refuses instead of overwriting a held slot
    del outs, host
    ring = HostTokenRing(dev, 512, slots=2)
    tok = torch.arange(8, device=dev, dtype=torch.int32)
    a = ring.take(tok)
    b = ring.take(tok)
    with pytest.raises(RuntimeError, match="overflow"):
        ring.take(tok)
    a[1].synchronize()
    assert a[0].tolist() == list(range(8))   # read: its slot is free again
    c = ring.take(tok * 2)
    c[1].synchronize()
    assert c[0].tolist() == [2 * i for i in range(8)] and b[0].tolist() == list(range(8))


def test_wait_kernel_deadline_reports_instead_of_hanging(gpu):
    """A device wait whose peer never arrives exits at its deadline and leaves its code."""
    from distributed_llm_inference import ops
    C = ops.native()
    words = C.HostWords(2)
    s = torch.cuda.Stream()
    C.wait_geq(words.dev_ptr(0), 1, 0.2, words.dev_ptr(1), 7, s.cuda_stream, 0)
    s.synchronize()
    assert words.get(1) == 7
    # satisfied wait: no code
    words.set(1, 0)
    words.set(0, 5)
    C.wait_geq(words.dev_ptr(0), 5, 5.0, words.dev_ptr(1), 9, s.cuda_stream, 0)
    s.synchronize()
    assert words.get(1) == 0


def test_signal_then_wait_orders_data(gpu):
    """signal() publishes data written before it on its stream; wait_geq() on another stream
    makes later work see it (the IPC transport's protocol in one process)."""
    from distributed_llm_inference import ops
    C = ops.native()
    dev = torch.device("cuda", 0)
    buf = C.IpcBuffer(1 << 20, 0)
    words = C.HostWords(1)
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    flag = buf.ptr + (1 << 20) - 256
    data = buf.view(0, [1024], torch.float32)
    out = torch.empty(1024, device=dev)
    for it in range(1, 6):
        src = torch.full((1024,), float(it), device=dev)
        torch.cuda.synchronize()
        with torch.cuda.stream(b):
            C.wait_geq(flag, it, 5.0, words.dev_ptr(0), 1, b.cuda_stream, 0)
            out.copy_(data)
        with torch.cuda.stream(a):
            torch.cuda._sleep(1000000)
            data.copy_(src)
            C.signal(flag, it, a.cuda_stream)
        b.synchronize()
        assert words.get(0) == 0
        assert torch.all(out == it)
    buf.close()


def test_device_marks_report_stream_progress(gpu):
    """The watchdog's per-stream device marks: a mark queued behind a spinning wait stays at the
    previous step until the wait is released; marks on other streams are unaffected."""
    import time
    from distributed_llm_inference import ops
    from distributed_llm_inference.runtime.streams import RankStreams
    from distributed_llm_inference.runtime.watchdog import OpTracker
    C = ops.native()
    dev = torch.device("cuda", 0)
    rs = RankStreams(dev, "dedicated")
    tr = OpTracker()
    tr.enable_device_marks(dev)
    flags = C.HostWords(2)
    try:
        tr.device_mark("recv", 0, rs.recv)
        tr.device_mark("compute", 0, rs.compute)
        rs.synchronize()
        assert tr.device_state()["recv"] == [0, 0]
        C.wait_geq(flags.dev_ptr(0), 1, 10.0, flags.dev_ptr(1), 1, rs.recv.cuda_stream, 0)
        tr.device_mark("recv", 1, rs.recv)
        tr.device_mark("compute", 1, rs.compute)
        rs.compute.synchronize()
        time.sleep(0.05)
        st = tr.device_state()
        assert st["compute"] == [1, 1] and st["recv"] == [1, 0], st
        flags.set(0, 1)
        rs.recv.synchronize()
        assert tr.device_state()["recv"] == [1, 1] and flags.get(1) == 0
    finally:
        flags.set(0, 1)
        torch.cuda.synchronize(dev)
        rs.close()
