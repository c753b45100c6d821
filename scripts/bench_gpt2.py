"""BASELINE config 1: GPT-2-small forward through distributed_llm_inference/models (plumbing).
Random-init GPT-2-small (124M) weights, synthetic prompts, greedy decoding; on the CPU by default
(the torch reference path; no GPU needed), or on the GPU with --device cuda (HIP kernels).

    python scripts/bench_gpt2.py [--device cpu|cuda] [--batch 8] [--prompt-len 64] [--new 32]
Prints one JSON line: output tokens/s, p50 per-token latency, prefill time.
"""
import argparse
import json
import os
import random
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

ap = argparse.ArgumentParser()
ap.add_argument("--device", default="cpu")
ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--prompt-len", type=int, default=64)
ap.add_argument("--new", type=int, default=32)
ap.add_argument("--threads", type=int, default=0, help="torch CPU threads (0 = torch default)")
a = ap.parse_args()

import torch  # noqa: E402
from distributed_llm_inference.config import CacheConfig, ServeConfig  # noqa: E402
from distributed_llm_inference.runtime.engine import EngineConfig, LLMEngine  # noqa: E402
from distributed_llm_inference.runtime.sequence import SamplingParams, Sequence  # noqa: E402

if a.threads:
    torch.set_num_threads(a.threads)
cfg = EngineConfig(model="gpt2", random_init=True, seed=0,
                   cache=CacheConfig(num_blocks=max(64, a.batch * 4), block_size=64),
                   serve=ServeConfig(max_batch_size=a.batch, max_num_batched_tokens=a.batch * a.prompt_len,
                                     max_seq_len=a.prompt_len + a.new + 8,
                                     use_graphs=a.device != "cpu", graph_batch_sizes=[a.batch]))
eng = LLMEngine("gpt2", device=a.device, cfg=cfg)
rng = random.Random(0)
prompts = [[rng.randrange(50257) for _ in range(a.prompt_len)] for _ in range(a.batch)]
eng.generate(prompts[:1], SamplingParams(max_tokens=2, ignore_eos=True))   # warm-up
seqs = [Sequence(p, SamplingParams(max_tokens=a.new, ignore_eos=True)) for p in prompts]
for s in seqs:
    eng.scheduler.add(s)
t0 = time.perf_counter()
first = None
while eng.pipeline.round():
    if first is None and all(len(s.output) > 0 for s in seqs):
        first = time.perf_counter()
eng.pipeline.drain()
if a.device != "cpu":
    torch.cuda.synchronize()
t1 = time.perf_counter()
lat = []
for s in seqs:
    tt = s.token_times
    lat += [(tt[i + 1] - tt[i]) * 1e3 for i in range(len(tt) - 1)]
toks = sum(len(s.output) for s in seqs)
decode_toks = toks - len(seqs)
print(json.dumps({
    "metric": "GPT-2-small generation (BASELINE config 1, plumbing)", "device": a.device,
    "batch": a.batch, "prompt_len": a.prompt_len, "new_tokens": a.new,
    "output_tokens_per_s": round(toks / (t1 - t0), 1),
    "decode_tokens_per_s": round(decode_toks / (t1 - (first or t0)), 1),
    "p50_token_latency_ms": round(statistics.median(lat), 2) if lat else None,
    "prefill_s": round((first or t1) - t0, 3), "threads": torch.get_num_threads(),
    "data": "synthetic prompts, random-init GPT-2-small weights"}))
