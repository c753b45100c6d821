"""Environment probe on the GPU box: hipBLASLt GEMM rates at decode/prefill shapes, fp8 scaled_mm, graphs."""
import time, torch, json, os, subprocess
out = {}
dev = torch.device("cuda:0")
p = torch.cuda.get_device_properties(0)
out["device"] = dict(name=p.name, gcn=getattr(p, "gcnArchName", ""), cus=p.multi_processor_count, mem_gb=p.total_memory / 2**30)
def bench(fn, iters=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters): fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters
res = {}
for (M, K, N) in [(1, 8192, 10240), (8, 8192, 10240), (64, 8192, 10240), (128, 8192, 10240), (256, 8192, 10240), (256, 8192, 57344), (256, 28672, 8192), (512, 8192, 57344), (2048, 8192, 10240), (8192, 8192, 8192), (256, 8192, 128256)]:
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
    t = bench(lambda: torch.nn.functional.linear(a, w))
    res[f"bf16_{M}x{K}x{N}"] = dict(ms=t * 1e3, tflops=2 * M * N * K / t / 1e12, gbps=(N * K * 2 + M * K * 2 + M * N * 2) / t / 1e9)
out["gemm"] = res
try:
    f8 = torch.float8_e4m3fn
    res8 = {}
    for (M, K, N) in [(64, 8192, 10240), (256, 8192, 10240), (256, 8192, 57344), (256, 28672, 8192), (8192, 8192, 8192)]:
        a = torch.randn(M, K, device=dev).to(f8)
        w = torch.randn(N, K, device=dev).to(f8)
        sa = torch.ones(M, 1, device=dev)
        sb = torch.ones(1, N, device=dev)
        fn = lambda: torch._scaled_mm(a, w.t(), scale_a=sa, scale_b=sb, out_dtype=torch.bfloat16)
        t = bench(fn)
        res8[f"fp8_rowwise_{M}x{K}x{N}"] = dict(ms=t * 1e3, tflops=2 * M * N * K / t / 1e12, gbps=(N * K + M * K) / t / 1e9)
        s1 = torch.ones((), device=dev)
        fn = lambda: torch._scaled_mm(a, w.t(), scale_a=s1, scale_b=s1, out_dtype=torch.bfloat16)
        t = bench(fn)
        res8[f"fp8_tensor_{M}x{K}x{N}"] = dict(ms=t * 1e3, tflops=2 * M * N * K / t / 1e12, gbps=(N * K + M * K) / t / 1e9)
    out["fp8"] = res8
except Exception as e:
    out["fp8_err"] = repr(e)
# graph capture of a linear
a = torch.randn(64, 8192, device=dev, dtype=torch.bfloat16); w = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    for _ in range(3): y = a @ w.t()
torch.cuda.synchronize()
with torch.cuda.graph(g):
    y = a @ w.t()
out["graph_ms"] = bench(lambda: g.replay()) * 1e3
# copy bandwidth
x = torch.empty(2**30, dtype=torch.uint8, device=dev); y = torch.empty_like(x)
t = bench(lambda: y.copy_(x))
out["copy_GBps"] = 2 * 2**30 / t / 1e9
print(json.dumps(out, indent=1))
os.makedirs("gpurun_out", exist_ok=True)
json.dump(out, open("gpurun_out/probe_env.json", "w"), indent=1)
