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
