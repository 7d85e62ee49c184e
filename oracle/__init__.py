"""CPU oracle for the AnoMod hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package, and only as the checker (or the timed CPU port); the
product path (the anomod package / libanomod.so) never touches it.

* ``spec``   — numpy / pure-Python restatements, each citing the reference
               lines it follows (small cases, and the JSON-level rules).
* ``native`` — ctypes binding of liboracle.so (plain C restatement of the
               integer edge aggregation, quantiles, EWMA/z and PageRank;
               fast enough for full-size parity runs and the CPU baseline).

Parity pinning: decode rules and the nearest-rank convention are pinned by
golden vectors produced by the reference's own code
(tests/golden/gen/make_goldens.py); EWMA/z by pandas 2.3.3 ``ewm``;
PageRank by networkx 3.4.2 ``pagerank``.  The edge table / histogram itself
has no reference implementation: it is pinned by the
reference-decoded parent/service columns plus this independent
restatement.
"""
