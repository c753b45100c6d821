"""Debug: multi-process (host-staged, shared GPU) pipeline vs in-process reference, per config."""
import multiprocessing as mp
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

PROMPTS = [list(range(3, 40)), [7, 8, 9], list(range(200, 330)), [11], [5, 5, 5, 5]]


def cfgs(world, mbs, graphs):
    from distributed_llm_inference.config import CacheConfig, ModelSpec, ServeConfig
    from distributed_llm_inference.runtime.engine import EngineConfig
    spec = ModelSpec(name="t", vocab_size=1000, hidden_size=256, intermediate_size=512,
                     num_layers=4, num_heads=8, num_kv_heads=2, head_dim=32, rope_theta=10000.0,
                     max_position_embeddings=4096)
    return spec, EngineConfig(model=spec, pp=world, seed=5, cache=CacheConfig(num_blocks=256, block_size=64),
                              serve=ServeConfig(max_batch_size=8, max_num_batched_tokens=512,
                                                max_seq_len=1024, num_micro_batches=mbs,
                                                use_graphs=graphs, graph_batch_sizes=[1, 2, 4, 8]))


def worker(rank, world, port, mbs, graphs, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DLI_SHARE_GPU="1",
                      DLI_TRANSPORT="host", DLI_TUNING_DIR="off")
    import torch.distributed as dist
    from distributed_llm_inference.runtime.engine import init_pipeline_rank
    from distributed_llm_inference.runtime.sequence import SamplingParams
    _, cfg = cfgs(world, mbs, graphs)
    role, obj = init_pipeline_rank(cfg)
    if role == "driver":
        out = obj.generate(PROMPTS, SamplingParams(max_tokens=6, ignore_eos=True))
        obj.stop()
        q.put([s.output for s in out])
    else:
        obj.run()
    dist.destroy_process_group()


def main():
    os.environ["DLI_TUNING_DIR"] = "off"
    from distributed_llm_inference.runtime.engine import LLMEngine
    from distributed_llm_inference.runtime.sequence import SamplingParams
    ctx = mp.get_context("spawn")
    for graphs in (False, True):
        for mbs in (1, 3):
            spec, cfg = cfgs(1, mbs, graphs)
            ref = [s.output for s in LLMEngine(spec, device="cuda:0", cfg=cfg).generate(
                PROMPTS, SamplingParams(max_tokens=6, ignore_eos=True))]
            spec, cfg2 = cfgs(2, mbs, graphs)
            loc2 = [s.output for s in LLMEngine(spec, device="cuda:0", cfg=cfg2).generate(
                PROMPTS, SamplingParams(max_tokens=6, ignore_eos=True))]
            q = ctx.Queue()
            s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
            ps = [ctx.Process(target=worker, args=(r, 2, port, mbs, graphs, q)) for r in range(2)]
            for p in ps:
                p.start()
            got = q.get(timeout=300)
            for p in ps:
                p.join(60)
            print(f"graphs={graphs} mbs={mbs}\n  ref  {ref}\n  loc2 {loc2}\n  mp2  {got}\n  "
                  f"match_loc={ref == loc2} match_mp={ref == got}", flush=True)


if __name__ == "__main__":
    main()
