"""Host-side logic of lib/sparse.py (no kernels): the raw fragments held as views of one buffer are read in place
by voxelize() (no per-call concatenation); anything else falls back to a copy."""
import numpy as np
import torch


def test_fragment_views_are_read_in_place():
    from lib.sparse import _adjacent_views, fragment_views
    r = np.random.RandomState(0)
    frags = [r.rand(n, 3).astype(np.float32) for n in (5, 1, 7)]
    views = fragment_views(frags, "cpu")
    assert [v.shape[0] for v in views] == [5, 1, 7]
    whole = _adjacent_views(views, "cpu")
    assert whole is not None and whole.data_ptr() == views[0].data_ptr()
    np.testing.assert_array_equal(whole.numpy(), np.concatenate(frags))


def test_non_adjacent_fragments_fall_back():
    from lib.sparse import _adjacent_views
    a = torch.arange(30.).reshape(10, 3)
    assert _adjacent_views([a[0:4], a[5:10]], "cpu") is None          # a gap
    assert _adjacent_views([a[4:10], a[0:4]], "cpu") is None          # out of order
    assert _adjacent_views([a[0:4].double(), a[4:10].double()], "cpu") is None
    assert _adjacent_views([], "cpu") is None


def test_adjacent_but_separate_storages_fall_back():
    """two tensors that sit side by side in memory but are NOT views of one storage (as separately allocated
    device tensors can be in the caching allocator): no in-place view (set_() on the first storage would resize it
    and leave the later fragments uninitialised); the copy path is taken"""
    from lib.sparse import _adjacent_views
    ba = bytearray(4 * 3 * 7)
    a = torch.frombuffer(ba, dtype=torch.float32, count=12, offset=0).reshape(4, 3)
    b = torch.frombuffer(ba, dtype=torch.float32, count=9, offset=48).reshape(3, 3)
    assert b.data_ptr() == a.data_ptr() + a.numel() * 4                     # adjacent ...
    assert a.untyped_storage().data_ptr() != b.untyped_storage().data_ptr()  # ... but two storages
    assert _adjacent_views([a, b], "cpu") is None
