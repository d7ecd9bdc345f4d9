"""The f16x2 scale cache's bookkeeping (lpgnn/fc.py _ScaleCache), on CPU tensors: entries keyed by the
base storage region (a view sliced afresh hits), invalidated by any in-place change of the base or a view
(the shared autograd version), never returned for a different region, dtype-free of the values."""
import gc

import torch

from lpgnn.fc import _ScaleCache


def test_views_of_one_region_share_an_entry():
    c = _ScaleCache()
    base = torch.randn(10, 8)
    c.put("row", base[:6], "s")
    assert c.lookup("row", base[:6]) == "s"          # a fresh view of the same rows
    assert c.lookup("col", base[:6]) is None          # the other kind
    assert c.lookup("row", base[:5]) is None          # another region
    assert c.lookup("row", base[1:7]) is None         # another offset
    assert c.lookup("row", base) is None              # the whole base is another operand


def test_in_place_change_invalidates():
    c = _ScaleCache()
    base = torch.randn(10, 8)
    v = base[:6]
    c.put("row", v, "s")
    base[8].add_(1.0)                                 # any write to the base bumps the shared version
    assert c.lookup("row", base[:6]) is None
    c.put("row", v, "t")
    v.mul_(2.0)                                       # and a write through the view
    assert c.lookup("row", v) is None


def test_freed_base_never_matches():
    c = _ScaleCache()
    t = torch.randn(4, 4)
    c.put("row", t, "s")
    key_id = id(t)
    del t
    gc.collect()
    u = torch.randn(4, 4)
    # even if the allocator hands out the same id, the weak reference to the old base is dead
    if id(u) == key_id:
        assert c.lookup("row", u) is None
    assert c.lookup("row", u) is None


def test_get_computes_once():
    c = _ScaleCache()
    t = torch.randn(3, 4)
    calls = []
    mk = lambda x: calls.append(1) or "v"  # noqa: E731
    assert c.get("col", t, mk) == "v" and c.get("col", t, mk) == "v"
    assert len(calls) == 1


def test_forget_drops_every_view_of_the_base():
    c = _ScaleCache()
    base = torch.randn(10, 8)
    other = torch.randn(10, 8)
    c.put("row", base[:6], "a")
    c.put("col", base, "b")
    c.put("row", other, "c")
    c.forget(base[6:])                                # any view names the whole base
    assert c.lookup("row", base[:6]) is None and c.lookup("col", base) is None
    assert c.lookup("row", other) == "c"
