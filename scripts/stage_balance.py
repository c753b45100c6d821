"""Per-stage decode time of the real PP=N layer ranges, measured on ONE GPU, with the LM head on
the last stage vs rotated over every rank (runtime/head.py).

Builds the N stage executors of Llama-3-70B in one process (in-process pipeline, all on one
MI355X), runs a few decode steps at B = 512, then times each stage's captured decode graph on its
own (HIP events around back-to-back replays) plus the rotating head's projection + sampling graph.
A pipeline runs at the pace of its slowest stage, so the balance that matters is max / mean of the
per-stage times: last-stage head = [s_0 .. s_(N-2), s_(N-1) + head]; rotating head =
[s_i + head / N], with the last stage's graph ending at the final norm.

    python scripts/stage_balance.py --pp 8 --batch 512      -> gpurun_out/stage_balance.json
"""
import argparse
import json
import os
import random
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-70b")
    ap.add_argument("--pp", type=int, default=8)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    from distributed_llm_inference.config import CacheConfig, ServeConfig, plan_stages, resolve_model
    from distributed_llm_inference.runtime.engine import EngineConfig, LLMEngine
    from distributed_llm_inference.runtime.executor import StepPlan
    from distributed_llm_inference.runtime.head import HeadRunner
    from distributed_llm_inference.runtime.sequence import SamplingParams, Sequence
    spec = resolve_model(a.model)
    B = a.batch
    cfg = EngineConfig(model=a.model, pp=a.pp, seed=0,
                       cache=CacheConfig(block_size=64, gpu_memory_utilization=0.92),
                       serve=ServeConfig(max_batch_size=B, max_num_batched_tokens=16384,
                                         num_micro_batches=1, max_seq_len=a.prompt_len + 120,
                                         graph_batch_sizes=[B]))
    eng = LLMEngine(a.model, pp=a.pp, device="cuda:0", cfg=cfg)
    drv = eng.pipeline
    rng = random.Random(0)
    seqs = [Sequence([rng.randrange(spec.vocab_size) for _ in range(a.prompt_len)],
                     SamplingParams(max_tokens=60, ignore_eos=True)) for _ in range(B)]
    for s in seqs:
        drv.sched.add(s)
    while any(len(s.output) == 0 for s in seqs):
        drv.round()
    for _ in range(4):
        drv.round()
    drv.barrier()

    def time_graph(fn):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            fn()
        e.record()
        e.synchronize()
        return s.elapsed_time(e) / a.reps

    exs = drv.executors
    stage_ms = []
    for ex in exs:   # the graphs replay the last staged decode step (same slots, same lengths)
        g = ex._graphs[B]
        stage_ms.append(time_graph(g.graph.replay))
    last = exs[-1]
    gn = last._capture(B, project=False)
    last_norm_ms = time_graph(gn.graph.replay)
    runner = HeadRunner(last.stage.head, last.device, B, True, [B])
    plan = StepPlan(1, 0, list(range(B)), [1] * B, sample_rows=list(range(B)),
                    temperature=[0.0] * B, top_k=[0] * B, top_p=[1.0] * B, seeds=[0] * B,
                    sample_pos=[0] * B)
    head_ms = time_graph(lambda: runner.run(plan, None))
    N = a.pp
    fixed = stage_ms
    rot = [t + head_ms / N for t in stage_ms[:-1]] + [last_norm_ms + head_ms / N]

    def bal(ts):
        return round(max(ts) / (sum(ts) / len(ts)), 4)

    res = dict(model=a.model, pp=N, batch=B, context=a.prompt_len,
               ranges_fixed_head=plan_stages(spec, N), ranges_rotating_head=plan_stages(
                   spec, N, head_rotation=True),
               ranges_measured=[[ex.stage.start, ex.stage.end] for ex in exs],
               stage_ms_fixed_head=[round(t, 3) for t in fixed],
               stage_ms_rotating_head=[round(t, 3) for t in rot],
               last_stage_to_norm_ms=round(last_norm_ms, 3), head_proj_sample_ms=round(head_ms, 3),
               max_over_mean_fixed=bal(fixed), max_over_mean_rotating=bal(rot),
               pipeline_pace_gain_pct=round(100 * (max(fixed) / max(rot) - 1), 2))
    print(json.dumps(res), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open("gpurun_out/stage_balance.json", "w"), indent=1)


if __name__ == "__main__":
    with torch.inference_mode():
        main()
