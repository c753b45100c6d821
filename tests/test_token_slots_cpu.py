"""HostTokenRing slot bookkeeping (runtime/streams.py SlotLedger / TokenSlot), host side: a slot
is held from take() until its consumer reads it (tolist), releases it, or drops the handle; a
hand-out onto a held slot raises instead of overwriting unread tokens."""
import gc

import pytest
import torch

from distributed_llm_inference.runtime.streams import SlotLedger, TokenSlot


def _take(ledger, vals):
    k = ledger.acquire()
    return TokenSlot(torch.tensor(vals, dtype=torch.int32), ledger, k)


def test_read_releases_and_overflow_raises():
    L = SlotLedger(2)
    a = _take(L, [1, 2])
    b = _take(L, [3])
    assert L.in_use() == 2
    with pytest.raises(RuntimeError, match="overflow"):
        _take(L, [4])
    assert a.tolist() == [1, 2] and L.in_use() == 1     # read: released
    c = _take(L, [5])                                   # reuses a's slot
    assert b.tolist() == [3] and c.tolist() == [5] and L.in_use() == 0


def test_derived_view_does_not_free_but_dropped_or_released_handles_do():
    L = SlotLedger(2)
    a = _take(L, [1, 2, 3])
    v = a.view[:2]          # a derived view alone never frees the slot ...
    b = _take(L, [4])
    with pytest.raises(RuntimeError, match="overflow"):
        _take(L, [5])
    del a                   # ... dropping the handle (an aborted step's result) does
    gc.collect()
    assert L.in_use() == 1 and v.tolist() == [1, 2]
    b.release()             # explicit release, then a read is still possible from the view
    assert L.in_use() == 0 and b.tolist() == [4]
