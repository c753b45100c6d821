"""hipGraph helpers.

Reference: ``make_inference_graphed_callable(callable, sample_args, num_warmup_iters=3)``
(/root/reference/distributed_llm_inference/utils/cuda.py:6-77), used there to capture tiny pieces of
the decode step (RoPE, RMSNorm).  On ROCm ``torch.cuda.CUDAGraph`` is a hipGraph.  Same signature
and behaviour (side-stream warmup, tensor-only args, static input copy on pointer change), with the
static-output aliasing hazard fixed: outputs are cloned by default, so a later replay
can never overwrite a result the caller still holds.  ``clone_outputs=False`` opts into the
zero-copy static-buffer contract.

The runtime does not use this per-op helper on its hot path; it captures the WHOLE per-stage
decode step per batch bucket (``StageExecutor._capture`` in ``runtime/executor.py``).
"""
from __future__ import annotations

import contextlib
import gc
from typing import Callable

import torch
from torch.utils._pytree import tree_flatten, tree_unflatten


_RNG_PRIMED: dict = {}


@contextlib.contextmanager
def capture_guard():
    """No Python garbage collection while a graph is being captured: ``torch.cuda.graph`` runs
    ``gc.collect()`` before capture begins, but an automatic collection triggered by the
    allocations DURING the capture can destroy an unrelated dead object whose destructor makes a
    stream-capture-illegal HIP call (freeing another graph's pool, destroying an event) and
    abort the process.  Collection resumes (and catches up) after the capture."""
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


def prime_graph_rng(device=None) -> None:
    """Create the device generator's graph-safe RNG state outside inference mode.

    ``capture_begin`` registers the default generator with the graph and lazily allocates its
    seed/offset tensors on first use. If that first capture runs under ``torch.inference_mode``
    (the runtime's decode graphs do) they become inference tensors, and every later capture
    OUTSIDE inference mode fails with "Inplace update to inference tensor". One empty capture
    with inference mode off makes them ordinary tensors; later in-place updates are then legal
    in both modes. The generator re-allocates that state whenever its set of registered graphs
    becomes empty, so the priming graph is kept alive for the life of the process."""
    dev = torch.device(device if device is not None else "cuda")
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if idx in _RNG_PRIMED:
        return
    with torch.inference_mode(False), torch.cuda.device(idx):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s), capture_guard():
            with torch.cuda.graph(g, stream=s):
                torch.empty(1, device=f"cuda:{idx}").fill_(0)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize(idx)
    _RNG_PRIMED[idx] = g


def make_inference_graphed_callable(callable: Callable, sample_args, num_warmup_iters: int = 3,
                                    clone_outputs: bool = True, pool=None) -> Callable:
    assert not isinstance(callable, torch.nn.Module), "pass a function, not an nn.Module"
    if torch.is_autocast_enabled() and torch.is_autocast_cache_enabled():
        raise RuntimeError("graph capture does not support the autocast cache; "
                           "set cache_enabled=False")
    flat, _ = tree_flatten(sample_args)
    if not all(isinstance(a, torch.Tensor) for a in flat):
        raise TypeError("sample_args must contain only tensors")
    static_inputs = tuple(flat)
    n_user = len(static_inputs)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(num_warmup_iters):
            callable(*sample_args)
    torch.cuda.current_stream().wait_stream(s)

    prime_graph_rng()
    graph = torch.cuda.CUDAGraph()
    with capture_guard(), torch.cuda.graph(graph, pool=pool):
        outputs = callable(*sample_args)
    flat_out, spec = tree_flatten(outputs)
    static_outputs = tuple(flat_out)

    def replay(*user_args):
        flat_args, _ = tree_flatten(user_args)
        if len(flat_args) != n_user:
            raise TypeError(f"expected {n_user} tensor args, got {len(flat_args)}")
        for dst, src in zip(static_inputs, flat_args):
            if dst.data_ptr() != src.data_ptr():
                dst.copy_(src)
        graph.replay()
        outs = tuple(o.clone() if clone_outputs else o.detach() for o in static_outputs)
        return tree_unflatten(list(outs), spec)

    replay.graph = graph  # type: ignore[attr-defined]
    return replay
