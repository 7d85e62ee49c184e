"""C ABI: the library loads, exports what include/anomod.h declares, and the
host-side (no-GPU) entry points behave.  No compute call needs a GPU here."""
import ctypes as C
import re

import numpy as np
import pytest

import anomod
from anomod import _lib as L
from conftest import ROOT


def _header_functions():
    text = (ROOT / "include" / "anomod.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(anomod_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    lib = anomod.lib()
    names = _header_functions()
    assert len(names) >= 30
    for n in names:
        assert hasattr(lib, n), n
    assert sorted(L.EXPORTED_SYMBOLS) == names


def test_abi_constants_match_header():
    text = (ROOT / "include" / "anomod.h").read_text()
    assert f"#define ANOMOD_HIST_BINS {L.HIST_BINS}" in text
    assert f"#define ANOMOD_ABI_VERSION {L.ABI_VERSION}" in text
    assert anomod.lib().anomod_abi_version() == L.ABI_VERSION


def test_hist_bin_matches_oracle():
    from oracle import spec
    lib = anomod.lib()
    rng = np.random.default_rng(3)
    for v in list(rng.integers(0, 2**32, 5000)) + [0, 63, 64, 65, 2**32 - 1]:
        assert lib.anomod_hist_bin(int(v)) == spec.hist_bin(int(v))
    lo, hi = C.c_uint32(), C.c_uint32()
    for b in range(L.HIST_BINS):
        assert lib.anomod_hist_bin_bounds(b, C.byref(lo), C.byref(hi)) == 0
        assert (lo.value, hi.value) == spec.hist_bounds(b)
    assert lib.anomod_hist_bin_bounds(L.HIST_BINS, C.byref(lo), C.byref(hi)) == L.EINVAL


def test_no_gpu_fails_loudly():
    if anomod.device_count_safe() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(anomod.AnomodError):
        anomod.Context(0)


def test_synth_services():
    sn = anomod.synth_services("SN")
    assert len(sn) == 12 and sn == sorted(sn) and "nginx-web-server" in sn
    tt = anomod.synth_services("TT")
    assert len(tt) == 46 and tt == sorted(tt) and "ts-order-service" in tt


def test_synth_host_generation_structure():
    spec_ = anomod.SynthSpec("SN", seed=20251103, p_orphan_ppm=2000)
    sp = anomod.synth_generate_host(spec_, 20000)
    assert sp.n_traces == 20000
    lens = np.diff(sp.trace_ptr)
    assert set(np.unique(lens).tolist()) == {7, 8, 20}
    frac = np.array([(lens == k).mean() for k in (7, 8, 20)])
    np.testing.assert_allclose(frac, [0.6, 0.3, 0.1], atol=0.02)  # mixed-workload.lua mix
    assert 8.4 < sp.n_spans / sp.n_traces < 8.8
    assert (sp.svc < 12).all()
    assert sp.span_id.min() > 0
    # roots: exactly one per trace (no orphan on the root span)
    first = sp.trace_ptr[:-1].astype(np.int64)
    assert (sp.parent_span_id[first] == 0).all()
    assert int((sp.parent_span_id == 0).sum()) == sp.n_traces
    assert 0.003 < (sp.flags & 1).mean() < 0.007
    # deterministic
    sp2 = anomod.synth_generate_host(spec_, 20000)
    assert (sp2.dur_us == sp.dur_us).all() and (sp2.span_id == sp.span_id).all()
    # shard field changes the data
    sp3 = anomod.synth_generate_host(spec_, 100, shard=1)
    assert not np.array_equal(sp3.span_id[:50], sp.span_id[:50])


def test_synth_fault_injection():
    base = anomod.synth_generate_host(anomod.SynthSpec("SN", seed=1), 5000)
    f = anomod.synth_generate_host(
        anomod.SynthSpec("SN", seed=1, fault_service="home-timeline-service"), 5000)
    k = base.services.index("home-timeline-service")
    m = base.svc == k
    assert (f.dur_us[m].astype(np.uint64) == base.dur_us[m].astype(np.uint64) * 8).all()
    assert (f.dur_us[~m] == base.dur_us[~m]).all()
    assert f.flags[m].mean() > 0.15


def test_span_set_shard_partition():
    sp = anomod.synth_generate_host(anomod.SynthSpec("TT", seed=3), 3000)
    parts = [sp.shard(4, r) for r in range(4)]
    assert sum(p.n_traces for p in parts) == sp.n_traces
    assert sum(p.n_spans for p in parts) == sp.n_spans
    for r, p in enumerate(parts):
        first = p.trace_ptr[:-1].astype(np.int64)
        assert ((p.trace_hash[first] % np.uint64(4)) == r).all()
