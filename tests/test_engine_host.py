"""Host-side logic of anomod.features (no GPU): the metric-series -> service
mapping, memoised per distinct label value, equals the plain rule "longest
service name contained in the series' joined label text, first in service
order on ties" on fuzzed label sets."""
import random

import anomod
from anomod import engine


def _plain(key, services):
    labels = key[1] if len(key) > 1 else ()
    text = " ".join(str(v) for _, v in labels)
    best = None
    for i, s in enumerate(services):
        if s and s in text and (best is None or len(s) > len(services[best])):
            best = i
    return best


def test_series_service_memo_equals_plain_rule():
    services = anomod.synth_services("TT") + ["ts-order", "order-service", "x", ""]
    rng = random.Random(7)
    values = (services + [s + "-7d9f-x" for s in services] +
              ["node1", "container_cpu", "ts-order-service-ts-preserve-service", "", 42])
    keys = [("m", tuple((f"l{j}", rng.choice(values)) for j in range(rng.randint(0, 4))))
            for _ in range(5000)]
    keys.append(("m",))
    memo: dict = {}
    for k in keys:
        want = _plain(k, services)
        assert engine._series_service(k, services, memo) == want
        assert engine._series_service(k, services) == want


def test_latency_shift_matches_edges_by_service_name():
    """The baseline run may have seen a different service set (services_discovered
    lists only the services its traces name): edges are matched by names, so a
    service absent from one run changes nothing for the others."""
    import numpy as np

    from anomod.spans import EdgeTable

    def table(services, edges):  # edges: {(parent or "ROOT", child): (count, p99)}
        t = EdgeTable.empty(services, with_hist=False)
        S = len(services)
        for (p, c), (n, p99) in edges.items():
            r = (S if p == "ROOT" else services.index(p)) * S + services.index(c)
            t.count[r], t.p99_us[r] = n, p99
        return t

    base = table(["a", "b", "d"], {("ROOT", "a"): (50, 100.0), ("a", "b"): (40, 10.0),
                                   ("a", "d"): (40, 7.0)})
    cur = table(["a", "b", "c"], {("ROOT", "a"): (50, 100.0), ("a", "b"): (40, 80.0),
                                  ("a", "c"): (40, 5.0)})
    shift = engine._latency_shift(cur, base)
    np.testing.assert_allclose(shift, [0.0, 3.0, 0.0])  # b: p99 x 8; c has no baseline edge
    same = engine._latency_shift(cur, cur)
    assert (same == 0).all()
