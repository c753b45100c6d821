

def test_tile_gemm_splits_every_split_gets_k_tiles():
    """A split count the tile kernels reject ((s - 1) * ceil(kt / s) >= kt, e.g. 16 k-tiles 7 ways)
    is never chosen: prefill of a 1024-hidden model at M = 1500 picked 7 for its QKV product."""
    from distributed_llm_inference import ops
    for M in (128, 512, 1500, 2048):
        for N in (256, 1024, 1536, 4096, 10240):
            for K in (256, 512, 1024, 2048, 8192, 28672):
                s = ops.tile_gemm_splits(M, N, K)
                if s:
                    kt = K * 2 // 128
                    assert (s - 1) * -(-kt // s) < kt, (M, N, K, s)
    assert ops.tile_gemm_splits(1500, 1536, 1024) != 7
