#!/usr/bin/env python3
"""Replay the edge kernel's chunking (<= 64 traces / <= 256 spans per wave
chunk, rows of 64 spans) on the host generator's spans and count the parent
scan's row-steps per chunk (a row waits for its slowest lane):
  fwd N      first-match forward scan from the trace start, N ids per step
  bidir F B  unique ids: F ids forward from the trace start + B ids backward
             from the span's own position per step
usage: python scripts/sim_parent_scan.py [SN|TT|LONG] [n_traces]"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"), str(ROOT)]
import anomod  # noqa: E402


def main():
    topo = sys.argv[1] if len(sys.argv) > 1 else "TT"
    nt = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    sp = anomod.synth_generate_host(anomod.SynthSpec(topo, seed=20251103, p_orphan_ppm=100), nt)
    ptr = sp.trace_ptr.astype(np.int64)
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

    def cost(nf, nb):
        tot = 0
        for t0, t1 in chunks:
            a, b = ptr[t0], ptr[t1]
            for r0 in range(a, b, 64):
                tot += max(steps(i, nf, nb) for i in range(r0, min(r0 + 64, b)))
        return tot / len(chunks)

    print(f"{topo}: {n / nt:.2f} spans/trace, {len(chunks)} chunks")
    for nf, nb in ((10, 0), (16, 0), (6, 4), (8, 8)):
        print(f"  {'fwd' if nb == 0 else 'bidir'} {nf}+{nb}: {cost(nf, nb):.2f} row-steps/chunk")


if __name__ == "__main__":
    main()
