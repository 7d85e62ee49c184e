#!/usr/bin/env python3
"""Replay the edge kernel's chunking (<= 64 traces / <= 256 spans per wave
chunk, rows of 64 spans) on the host generator's spans and count the parent
scan's row-steps per chunk (a row waits for its slowest lane):
  fwd N      first-match forward scan from the trace start, N ids per step
  bidir F B  unique ids: F ids forward from the trace start + B ids backward
             from the span's own position per step
usage: python scripts/experiments/sim_parent_scan.py [SN|TT|LONG] [n_traces] [shuffled]
(shuffled: the spans of every trace in a random order first)"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"), str(ROOT)]
import anomod  # noqa: E402


def main():
    topo = sys.argv[1] if len(sys.argv) > 1 else "TT"
    nt = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    sp = anomod.synth_generate_host(anomod.SynthSpec(topo, seed=20251103, p_orphan_ppm=100), nt)
    ptr = sp.trace_ptr.astype(np.int64)
    if len(sys.argv) > 3 and sys.argv[3].startswith("shuf"):
        rng = np.random.default_rng(1)
        order = np.concatenate([a + rng.permutation(b - a) for a, b in zip(ptr[:-1], ptr[1:])])
        sp = sp.take(order, sp.trace_ptr)
    chunks, t = [], 0
    while t < nt:
        a, k = ptr[t], 0
        while t + k < nt and k < 64 and ptr[t + k + 1] - a <= 256:
            k += 1
        k = max(k, 1)
        chunks.append((t, t + k))
        t += k
    n = sp.n_spans
    par = np.full(n, -1)  # -1 root, -2 not found, else position of the first match
    ta, tb = np.zeros(n, np.int64), np.zeros(n, np.int64)
    for t in range(nt):
        a, b = ptr[t], ptr[t + 1]
        first = {}
        for i in range(a, b):
            first.setdefault(int(sp.span_id[i]), i)
        for i in range(a, b):
            p = int(sp.parent_span_id[i])
            ta[i], tb[i] = a, b
            par[i] = first.get(p, -2) if p else -1

    def steps(i, nf, nb):
        if par[i] == -1:
            return 0
        if par[i] == -2:
            return -(-(tb[i] - ta[i]) // nf)
        f = (par[i] - ta[i]) // nf + 1
        if nb == 0 or par[i] >= i:
            return f
        return min(f, (i - 1 - par[i]) // nb + 1)

    def steps_meet(i, nf, nb):
        """nf forward from the trace start + nb backward from i - 1 until the two
        meet ([a, i) covered), then nf + nb forward (chunk.h find_parent_bidir)."""
        if par[i] == -1:
            return 0
        a, b, q = ta[i], tb[i], par[i]
        f, g, k = a, i - 1, 0
        while True:
            k += 1
            if f <= g:
                gb = max(a, g - nb + 1)
                if f <= q < f + nf or gb <= q <= g:
                    return k
                f += nf
                g -= nb
            else:
                if f <= q < f + nf + nb:
                    return k
                f += nf + nb
            if f >= b:
                return k

    def steps_adj(i, nf, nb):
        """unique ids: the span just before (one read) settles it, else nf forward
        per step from the trace start"""
        if par[i] == -1:
            return 0
        if par[i] == i - 1:
            return 1
        return steps(i, nf, 0) + 1

    def steps_first(i, nf, nb):
        """unique ids: one bidirectional step (nf forward from the trace start, nb
        back from i - 1), then nf + nb forward per step"""
        if par[i] == -1:
            return 0
        a, b, q = ta[i], tb[i], par[i]
        if a <= q < a + nf or max(a, i - nb) <= q < i:
            return 1
        if q < 0:
            return 1 + -(-(b - a - nf) // (nf + nb))
        return 1 + (q - a - nf) // (nf + nb) + 1

    def cost(nf, nb, fn=None):
        fn = fn or steps
        tot = 0
        for t0, t1 in chunks:
            a, b = ptr[t0], ptr[t1]
            for r0 in range(a, b, 64):
                tot += max(fn(i, nf, nb) for i in range(r0, min(r0 + 64, b)))
        return tot / len(chunks)

    def cost_queue(nf, nb):
        """each lane works through its own spans of the chunk (positions l,
        l + 64, ...) one lookup after another; the wave steps until every
        lane's queue is empty: max over lanes of the lane's summed steps"""
        tot = 0
        for t0, t1 in chunks:
            a, b = ptr[t0], ptr[t1]
            tot += max(sum(steps(i, nf, nb) for i in range(a + l, b, 64)) for l in range(64))
        return tot / len(chunks)

    print(f"{topo}: {n / nt:.2f} spans/trace, {len(chunks)} chunks")
    import os
    splits = [tuple(int(x) for x in t.split("+")) for t in os.environ.get("SPLITS", "10+0 6+4").split()]
    for nf, nb in splits:
        print(f"  {'fwd' if nb == 0 else 'bidir'} {nf}+{nb}: {cost(nf, nb):.2f} row-steps/chunk")
    if os.environ.get("QUEUE"):
        for nf, nb in splits:
            print(f"  per-lane queue {nf}+{nb}: {cost_queue(nf, nb):.2f} row-steps/chunk")
    if os.environ.get("SIM_ALL"):
        for nf, nb in ((6, 4), (8, 2)):
            print(f"  bidir-meet {nf}+{nb}: {cost(nf, nb, steps_meet):.2f} row-steps/chunk")
        for nf, nb in ((6, 4), (8, 2), (4, 6)):
            print(f"  first bidir {nf}+{nb}, then fwd: {cost(nf, nb, steps_first):.2f} row-steps/chunk")


if __name__ == "__main__":
    main()
