"""The C grouping restatement (oracle_group_by_trace, timed as the ungrouped
leg's CPU baseline) equals spec.group_by_trace (numpy stable argsort of
mix64) on random, colliding and degenerate hash columns, for any thread count."""
import numpy as np
import pytest

from oracle import native, spec


def _hashes(kind, rng, n):
    if kind == "random":
        return rng.integers(0, 2**64, n, dtype=np.uint64)
    if kind == "few":  # long traces: few distinct hashes, interleaved
        return rng.integers(0, 50, n).astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    if kind == "traces":  # ~9 spans per trace
        return rng.integers(0, 2**64, max(1, n // 9), dtype=np.uint64)[rng.integers(0, max(1, n // 9), n)]
    return np.zeros(n, np.uint64)  # one trace


@pytest.mark.parametrize("kind", ["random", "few", "traces", "one"])
@pytest.mark.parametrize("n,threads", [(0, 4), (1, 1), (7, 3), (5000, 1), (200_000, 8)])
def test_group_by_trace_c_equals_numpy(kind, n, threads):
    rng = np.random.default_rng(n + threads)
    h = _hashes(kind, rng, n)
    o_ref, t_ref = spec.group_by_trace(h)
    o, t = native.group_by_trace(h, threads)
    np.testing.assert_array_equal(o, o_ref)
    np.testing.assert_array_equal(t, t_ref)
