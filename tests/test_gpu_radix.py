"""The hand-written onesweep radix sort (csrc/radix.hip, mvr_radix_sort_pairs) against numpy's stable argsort:
sizes around the 4096-key tile (empty, one key, a partial tile, exact tiles, many tiles), few distinct keys (long
runs of equal keys: stability across waves, tiles and the look-back), bit widths that are not a multiple of the
8-bit digit (the high bits above `bits` are ignored), caller-given values, and the kernel maps' real key shape
(27-bit offset masks above fragment + Morton bits, 2 M keys)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _sort(gpu, keys, bits, vals=None):
    import torch
    from lib import _native as N
    L = N.lib()
    n = len(keys)
    k = torch.from_numpy(keys.view(np.int64)).to(gpu)
    v = torch.from_numpy(vals).to(gpu) if vals is not None else None
    out = torch.full((max(n, 1),), -7, dtype=torch.int32, device=gpu)
    ws = torch.empty(L.mvr_radix_sort_pairs_bytes(n), dtype=torch.uint8, device=gpu)
    N.check(L.mvr_radix_sort_pairs(N.ptr(k), N.ptr(v), n, bits, N.ptr(out), N.ptr(ws), ws.numel(), N.stream()),
            "mvr_radix_sort_pairs")
    return out[:n].cpu().numpy()


def _ref(keys, bits):
    m = keys & np.uint64((1 << bits) - 1) if bits < 64 else keys
    return np.argsort(m, kind="stable").astype(np.int32)


@pytest.mark.parametrize("n", [0, 1, 63, 4095, 4096, 4097, 3 * 4096 + 17, 200003])
@pytest.mark.parametrize("bits,distinct", [(64, None), (59, 7), (13, None), (8, 3), (1, None)])
def test_radix_sort_equals_stable_argsort(gpu, n, bits, distinct):
    rng = np.random.default_rng(n + bits)
    if distinct:
        pool = rng.integers(0, 2 ** 63, distinct, dtype=np.uint64)
        keys = pool[rng.integers(0, distinct, n)]
    else:
        keys = rng.integers(0, 2 ** 63, n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, n, dtype=np.uint64)
    got = _sort(gpu, keys, bits)
    np.testing.assert_array_equal(got, _ref(keys, bits))


def test_radix_sort_values_and_kernel_map_key_shape(gpu):
    """2 M keys shaped like the batched kernel-map keys (map index << 59 | 27-bit mask << 32 | fragment + Morton):
    skewed masks (a few classes hold most rows), caller values carried through"""
    rng = np.random.default_rng(1)
    n = 2_000_000
    maps = np.sort(rng.integers(0, 10, n)).astype(np.uint64)
    masks = np.where(rng.random(n) < 0.7, rng.integers(0, 12, n), rng.integers(0, 1 << 27, n)).astype(np.uint64)
    lo = rng.integers(0, 1 << 32, n, dtype=np.uint64)
    keys = maps << np.uint64(59) | masks << np.uint64(32) | lo
    vals = rng.integers(-2 ** 31, 2 ** 31 - 1, n).astype(np.int32)
    got = _sort(gpu, keys, 63, vals)
    np.testing.assert_array_equal(got, vals[_ref(keys, 63)])
