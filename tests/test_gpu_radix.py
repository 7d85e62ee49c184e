"""GPU: the hand-written stable LSD radix sort (csrc/radix.hip) under the exact
order-statistic paths — the exact per-edge quantiles (§8a a11) and the API
value summary (§8f row 3), both restating the reference's sorted(x)[int(n*q)]
(monitor_http_responses.py:180-190).  Checked against numpy's stable sort:
ragged sizes around the 4096-key tile, every bit range the callers use,
duplicate-heavy keys, constant digits (skipped passes), and stability (keys
equal in the sorted bits keep their input order)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [1, 2, 63, 4095, 4096, 4097, 100_003, 2_000_000])
def test_sort_full_keys(ctx, n):
    rng = np.random.default_rng(n)
    k = rng.integers(0, 2**64, n, dtype=np.uint64)
    got, passes = ctx.sort_u64(k)
    np.testing.assert_array_equal(got, np.sort(k))
    assert passes == 8 or n < 3


@pytest.mark.parametrize("end_bit", [9, 16, 40, 44, 63])
def test_sort_bit_ranges_and_duplicates(ctx, end_bit):
    rng = np.random.default_rng(end_bit)
    n = 300_001
    # edge<<32 | dur style: few distinct high parts, heavy duplicates
    k = rng.integers(0, 2**min(end_bit, 20), n, dtype=np.uint64)
    if end_bit > 32:
        k = (rng.integers(0, 2**(end_bit - 32), n, dtype=np.uint64) << np.uint64(32)) | (k & 0xFFFF)
    got, _ = ctx.sort_u64(k, 0, end_bit)
    np.testing.assert_array_equal(got, np.sort(k))


def test_sort_is_stable_on_the_sorted_bits(ctx):
    """Sort by bits [32, 48) only: keys with equal bits 32..47 keep their
    input order (the low 32 bits carry the input position)."""
    rng = np.random.default_rng(3)
    n = 500_000
    hi = rng.integers(0, 300, n, dtype=np.uint64)
    k = (hi << np.uint64(32)) | np.arange(n, dtype=np.uint64)
    got, passes = ctx.sort_u64(k, 32, 48)
    order = np.argsort(hi, kind="stable")
    np.testing.assert_array_equal(got, k[order])
    assert passes == 2  # bits 32-39 and 40-47 vary (hi < 300 < 2^9)


def test_sort_skips_constant_digits(ctx):
    rng = np.random.default_rng(4)
    k = (np.uint64(0xABCD) << np.uint64(40)) | rng.integers(0, 256, 50_000, dtype=np.uint64)
    got, passes = ctx.sort_u64(k)
    np.testing.assert_array_equal(got, np.sort(k))
    assert passes == 1
    same, passes = ctx.sort_u64(np.full(10_000, 7, np.uint64))
    assert passes == 0 and (same == 7).all()
