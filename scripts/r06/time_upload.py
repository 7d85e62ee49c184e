#!/usr/bin/env python3
"""Host -> device copy rates the upload pipeline can reach: hipHostRegister /
Unregister of pageable numpy buffers, DMA from registered and from
hipHostMalloc'd memory over 1 / 4 / 8 streams, and pageable hipMemcpyAsync.

  python scripts/r06/time_upload.py [MiB]
"""
import ctypes as C
import json
import sys
import time

import numpy as np

mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
nbytes = mib << 20
hip = C.CDLL("libamdhip64.so")
vp = C.c_void_p
hip.hipMalloc.argtypes = [C.POINTER(vp), C.c_size_t]
hip.hipHostMalloc.argtypes = [C.POINTER(vp), C.c_size_t, C.c_uint]
hip.hipHostRegister.argtypes = [vp, C.c_size_t, C.c_uint]
hip.hipHostUnregister.argtypes = [vp]
hip.hipMemcpyAsync.argtypes = [vp, vp, C.c_size_t, C.c_int, vp]
hip.hipStreamCreateWithFlags.argtypes = [C.POINTER(vp), C.c_uint]
hip.hipStreamSynchronize.argtypes = [vp]
H2D = 1


def ms(t0):
    return round((time.perf_counter() - t0) * 1e3, 3)


d = vp()
assert hip.hipMalloc(C.byref(d), nbytes) == 0
streams = []
for _ in range(8):
    s = vp()
    assert hip.hipStreamCreateWithFlags(C.byref(s), 1) == 0
    streams.append(s)


def dma(src, ns, piece=8 << 20):
    t0 = time.perf_counter()
    off, k = 0, 0
    while off < nbytes:
        n = min(piece, nbytes - off)
        assert hip.hipMemcpyAsync(vp(d.value + off), vp(src + off), n, H2D, streams[k % ns]) == 0
        off += n
        k += 1
    for s in streams[:ns]:
        hip.hipStreamSynchronize(s)
    el = time.perf_counter() - t0
    return round(el * 1e3, 3), round(nbytes / el / 1e9, 2)


out = {"MiB": mib}
a = np.ones(nbytes // 8, np.uint64)  # pageable, touched
src = a.ctypes.data
for rep in range(3):
    t0 = time.perf_counter()
    rc = hip.hipHostRegister(vp(src), nbytes, 0)
    reg = ms(t0)
    r = {"register_ms": reg, "rc": rc}
    for ns in (1, 4, 8):
        r[f"registered_dma_{ns}"] = dma(src, ns)
    t0 = time.perf_counter()
    hip.hipHostUnregister(vp(src))
    r["unregister_ms"] = ms(t0)
    out[f"register_{rep}"] = r
    print(json.dumps(r), flush=True)
p = vp()
t0 = time.perf_counter()
assert hip.hipHostMalloc(C.byref(p), nbytes, 0) == 0
out["hostmalloc_ms"] = ms(t0)
C.memset(p, 1, nbytes)
for ns in (1, 4, 8):
    out[f"pinned_dma_{ns}"] = [dma(p.value, ns) for _ in range(2)]
for piece in (32 << 20, 128 << 20):
    out[f"pinned_dma_8_piece{piece >> 20}M"] = dma(p.value, 8, piece)
out["pageable_dma_1"] = [dma(src, 1) for _ in range(2)]
print(json.dumps(out), flush=True)
