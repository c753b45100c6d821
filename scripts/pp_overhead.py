"""Per-stage overhead of the pipeline runtime, measured on ONE GPU.

Runs the same decode workload through an in-process pipeline of P stages (all on one GPU, so the
stages execute back to back) and through a single stage.  The difference in step time is what
splitting the model costs per stage: per-stage metadata upload, one hipGraph launch per stage,
the hidden-state hand-off copy and the smaller per-graph kernel chains.  At PP=8 on 8 GPUs each
stage's share of the step is ~1/8 of the single-stage time, so this overhead / 8 must stay small.

    python scripts/pp_overhead.py --model llama-3-70b --pp 8 --batch 512 --steps 6
"""
import argparse
import json
import os
import random
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(model, pp, batch, steps, prompt_len):
    from distributed_llm_inference.config import CacheConfig, ServeConfig, resolve_model
    from distributed_llm_inference.runtime.engine import EngineConfig, LLMEngine
    from distributed_llm_inference.runtime.sequence import SamplingParams, Sequence
    spec = resolve_model(model)
    cfg = EngineConfig(model=model, pp=pp, seed=0,
                       cache=CacheConfig(block_size=64, gpu_memory_utilization=0.92),
                       serve=ServeConfig(max_batch_size=batch, max_num_batched_tokens=16384,
                                         num_micro_batches=1, max_seq_len=prompt_len + steps + 80,
                                         graph_batch_sizes=[batch]))
    eng = LLMEngine(model, pp=pp, device="cuda:0", cfg=cfg)
    drv = eng.pipeline
    rng = random.Random(0)
    seqs = [Sequence([rng.randrange(spec.vocab_size) for _ in range(prompt_len)],
                     SamplingParams(max_tokens=steps + 40, ignore_eos=True)) for _ in range(batch)]
    for s in seqs:
        drv.sched.add(s)
    while any(len(s.output) == 0 for s in seqs):
        drv.round()
    for _ in range(3):
        drv.round()
    drv.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        drv.round()
    drv.barrier()
    ms = (time.perf_counter() - t0) / steps * 1e3
    del eng, drv
    torch.cuda.empty_cache()
    return ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-70b")
    ap.add_argument("--pp", type=int, default=8)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--prompt-len", type=int, default=128)
    a = ap.parse_args()
    one = run(a.model, 1, a.batch, a.steps, a.prompt_len)
    many = run(a.model, a.pp, a.batch, a.steps, a.prompt_len)
    res = dict(model=a.model, batch=a.batch, pp=a.pp, step_ms_pp1=round(one, 2),
               step_ms_ppN_one_gpu=round(many, 2),
               overhead_ms_per_stage=round((many - one) / a.pp, 3),
               overhead_pct_of_stage_at_ppN=round(100 * (many - one) / one, 2))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
