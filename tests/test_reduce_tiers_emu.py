"""The sharded reduce's block-tier ordering on the CPU (csrc/kernels/dist.hip; no GPU).

A block tier (lead_block_tier) sums one lead's partials by trail in LDS, keeps the trails whose
sum lies in [min, max] (KmerTable.calcDispatchData's filter, :155-187) and writes them back in
trail order: up to 512 kept by counting ranks, past that by a bitonic network over the next
power of two, padded with 0xFFFFFFFF keys.  This emulates that network stage by stage, with the
kernel's index rule (pair t of a stage: i = 2t - (t & (stride - 1)), partner i + stride,
ascending where (i & size) == 0), vectorised over t, and checks the written segment against a
plain sort of the kept entries.  The GPU tests test_gpu_parity.py::test_virtual_shards_reduce_tiers
check the kernels themselves."""
import numpy as np
import pytest

EMPTY = 0xFFFFFFFF


def bitonic_like_kernel(keys, vals):
    """dist.hip's network: P = the next power of two >= k (at least 64), pads last."""
    k = len(keys)
    P = 64
    while P < k:
        P <<= 1
    a = np.full(P, EMPTY, dtype=np.uint64)
    b = np.zeros(P, dtype=np.uint64)
    a[:k] = keys
    b[:k] = vals
    t = np.arange(P // 2, dtype=np.int64)
    size = 2
    while size <= P:
        stride = size >> 1
        while stride:
            i = 2 * t - (t & (stride - 1))
            i2 = i + stride
            up = (i & size) == 0
            swap = (a[i] > a[i2]) == up
            ai, bi = a[i].copy(), b[i].copy()
            a[i] = np.where(swap, a[i2], a[i])
            b[i] = np.where(swap, b[i2], b[i])
            a[i2] = np.where(swap, ai, a[i2])
            b[i2] = np.where(swap, bi, b[i2])
            stride >>= 1
        size <<= 1
    return a[:k], b[:k]


def block_tier(trails, counts, min_c, max_c):
    """One lead through a block tier: sum by trail, filter, order by trail."""
    u, inv = np.unique(trails, return_inverse=True)
    sums = np.bincount(inv, weights=counts).astype(np.int64)
    keep = (sums >= min_c) & (sums <= max_c)
    kk, kc = u[keep], sums[keep]
    rng = np.random.default_rng(len(kk))
    order = rng.permutation(len(kk))  # the LDS table's order is a hash order, not the trails'
    kk, kc = kk[order], kc[order]
    if len(kk) > 512:
        return bitonic_like_kernel(kk, kc)
    r = np.array([(kk < e).sum() for e in kk], dtype=np.int64)  # the counting rank
    out_k = np.empty_like(kk)
    out_c = np.empty_like(kc)
    out_k[r] = kk
    out_c[r] = kc
    return out_k, out_c


@pytest.mark.parametrize("k", [1, 63, 64, 65, 513, 1000, 3072, 4096, 6000, 12288])
def test_bitonic_network_sorts_with_pads(k):
    rng = np.random.default_rng(k)
    keys = rng.choice(2_000_000, size=k, replace=False).astype(np.uint64)
    vals = rng.integers(1, 1000, size=k).astype(np.uint64)
    a, b = bitonic_like_kernel(keys, vals)
    order = np.argsort(keys)
    np.testing.assert_array_equal(a, keys[order])
    np.testing.assert_array_equal(b, vals[order])


@pytest.mark.parametrize("partners,min_c", [(300, 2), (3000, 2), (9000, 3), (12288, 1)])
def test_block_tier_output_is_trail_ordered_kept_sums(partners, min_c):
    rng = np.random.default_rng(partners)
    trails = rng.choice(5_000_000, size=partners, replace=False)
    # each partner's collisions arrive as partials from up to 8 owners
    reps = rng.integers(1, 9, size=partners)
    t = np.repeat(trails, reps)
    c = rng.integers(1, 3, size=len(t))
    got_k, got_c = block_tier(t, c, min_c, 10_000)
    sums = {}
    for x, y in zip(t.tolist(), c.tolist()):
        sums[x] = sums.get(x, 0) + y
    want = sorted((x, y) for x, y in sums.items() if min_c <= y <= 10_000)
    assert len(want) > 0
    np.testing.assert_array_equal(got_k, [x for x, _ in want])
    np.testing.assert_array_equal(got_c, [y for _, y in want])
