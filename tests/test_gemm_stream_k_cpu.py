"""CPU model of the tile GEMM's stream-K tail decomposition (csrc/kernels/gemm_tile.hip, SkArgs):
the same integer math as the kernel, checked for exact coverage and a consistent hand-off graph."""
import pytest


def sk_plan(tiles, kt, cus):
    """Per stream-K workgroup: list of (tile, k0, k1, kind, preds) in execution order, as the
    kernel derives them (kind: 'publish' | 'finish' | 'full')."""
    n_dp = tiles // cus * cus
    total = (tiles - n_dp) * kt
    plan = []
    for lid in range(cus):
        lo, hi = total * lid // cus, total * (lid + 1) // cus
        first_t = lo // kt
        nseg = (hi - 1) // kt - first_t + 1
        segs = []
        for seg in range(nseg):
            t = first_t + (0 if nseg == 1 else nseg - 1 if seg == 0 else 0 if seg == nseg - 1 else seg)
            tk0 = t * kt
            s0, s1 = max(lo, tk0), min(hi, tk0 + kt)
            publish = s1 < tk0 + kt
            finish = not publish and s0 > tk0
            preds = []
            if finish:
                for p in range(lid - 1, -1, -1):
                    preds.append(p)
                    if total * p // cus <= tk0:
                        break
            kind = "publish" if publish else "finish" if finish else "full"
            segs.append((n_dp + t, s0 - tk0, s1 - tk0, kind, preds))
        plan.append(segs)
    return n_dp, plan


@pytest.mark.parametrize("tiles,kt", [(448, 128), (448, 16), (384, 4), (288, 32), (260, 64),
                                      (300, 7), (511, 3), (257, 1000)])
def test_stream_k_tail_covers_every_k_tile_once(tiles, kt):
    cus = 256
    if (tiles - tiles // cus * cus) * kt < cus:
        pytest.skip("launcher refuses: fewer k-tiles than stream-K workgroups")
    n_dp, plan = sk_plan(tiles, kt, cus)
    cover = {}
    published = {}
    for lid, segs in enumerate(plan):
        kinds = [s[3] for s in segs]
        # at most one publish (run first) and one finish (run last); nothing waits before publishing
        assert kinds.count("publish") <= 1 and kinds.count("finish") <= 1
        if "publish" in kinds:
            assert kinds[0] == "publish"
        if "finish" in kinds:
            assert kinds[-1] == "finish"
        for tile, k0, k1, kind, preds in segs:
            assert 0 <= k0 < k1 <= kt
            for k in range(k0, k1):
                assert (tile, k) not in cover
                cover[(tile, k)] = lid
            if kind == "publish":
                published[lid] = tile
    assert len(cover) == (tiles - n_dp) * kt
    # every tile has exactly one writer of its output (full or finish); a finisher's predecessor
    # chain is exactly the set of workgroups that published a piece of that tile
    writers = {}
    for lid, segs in enumerate(plan):
        for tile, k0, k1, kind, preds in segs:
            if kind == "publish":
                continue
            assert tile not in writers
            writers[tile] = lid
            owners = {cover[(tile, k)] for k in range(kt)} - {lid}
            assert set(preds) == owners
            assert all(published.get(p) == tile for p in preds)
            assert all(p < lid for p in preds)
    assert sorted(writers) == list(range(n_dp, tiles))
    assert set(published) == {p for segs in plan for s in segs for p in s[4]}
