"""GPU parity: EWMA/z kernel vs pandas golden + C oracle; PageRank vs
networkx golden + C oracle; the load -> features -> rank surface."""
import numpy as np
import pytest

import anomod
from anomod import _lib as L
from oracle import native, spec

pytestmark = pytest.mark.gpu

# z is computed in f32 from f64 state on the GPU (f64 in the oracle): 1e-5 rel.
Z_RTOL, Z_ATOL = 1e-5, 1e-5


def test_ewma_matches_pandas_golden(ctx, golden):
    g = np.load(golden / "ewma_pandas.npz")
    X, M, V, a = g["X"], g["mean"], g["var"], float(g["alpha"])
    W, eps = 60, 1e-12
    Z = ctx.ewma_z(X, a, W, eps)
    np.testing.assert_allclose(Z, spec.window_scores_from_state(X, M, V, W, eps),
                               rtol=Z_RTOL, atol=Z_ATOL)


@pytest.fixture(params=[1, 2, 3], ids=["sequential_tiles", "time_parallel", "sequential_rows"])
def ewma_mode(request, monkeypatch):
    """Run a test under every EWMA kernel (ANOMOD_EWMA_MODE, read per call)."""
    monkeypatch.setenv("ANOMOD_EWMA_MODE", str(request.param))
    return request.param


@pytest.mark.parametrize("T,S,W", [(60, 1, 60), (600, 1000, 60), (4800, 77, 16), (256, 5000, 1),
                                   (960, 130, 96), (1200, 70, 150), (1010, 90, 10),
                                   (7, 3, 7)])
def test_ewma_matches_oracle(ctx, ewma_mode, T, S, W):
    rng = np.random.default_rng(T + S)
    X = (rng.uniform(0, 1e4, S) + rng.uniform(0.1, 10, S) * rng.standard_normal((T, S)))
    X = X.astype(np.float32)
    X[rng.random((T, S)) < 0.01] = np.nan
    a = 2.0 / (W + 1) if W > 1 else 0.3
    np.testing.assert_allclose(ctx.ewma_z(X, a, W), native.ewma_z(X, a, W),
                               rtol=Z_RTOL, atol=Z_ATOL)


def test_ewma_streaming_chunks_equal_one_pass(ctx, ewma_mode):
    rng = np.random.default_rng(1)
    T, S, W = 1200, 300, 60
    X = (100 + rng.standard_normal((T, S))).astype(np.float32)
    one = ctx.ewma_z(X, 2 / 61, W)
    ser = anomod.DeviceSeries(ctx, T // 2, S)
    ser.upload(X[: T // 2])
    z1 = ser.ewma_z(2 / 61, W)
    ser.upload(X[T // 2:])
    z2 = ser.ewma_z(2 / 61, W)
    np.testing.assert_array_equal(np.concatenate([z1, z2]), one)
    ser.free()


@pytest.mark.parametrize("T,S,W,seg", [(4800, 300, 60, 960), (4800, 300, 60, 2000),
                                       (3136, 200, 7, 448), (1000, 65, 1, 64)])
def test_ewma_time_segments_equal_one_launch(ctx, monkeypatch, T, S, W, seg):
    """The sequential tiled kernel runs a long T as launches of a multiple of
    lcm(W, 64) steps (ANOMOD_EWMA_SEG rounded down to one), the state carried
    through HBM: bit-equal to one launch, with NaN runs and late starts."""
    monkeypatch.setenv("ANOMOD_EWMA_MODE", "1")
    rng = np.random.default_rng(T + W)
    X = (100 + rng.standard_normal((T, S))).astype(np.float32)
    X[: T // 3, : S // 4] = np.nan
    X[rng.random((T, S)) < 0.05] = np.nan
    a = 2.0 / (W + 1) if W > 1 else 0.3
    monkeypatch.setenv("ANOMOD_EWMA_SEG", "0")
    one = ctx.ewma_z(X, a, W)
    monkeypatch.setenv("ANOMOD_EWMA_SEG", str(seg))
    np.testing.assert_array_equal(ctx.ewma_z(X, a, W), one)
    np.testing.assert_allclose(one, native.ewma_z(X, a, W), rtol=Z_RTOL, atol=Z_ATOL)


def test_ewma_time_parallel_nan_runs_and_fresh_start(ctx, monkeypatch):
    """Leading all-NaN sub-chunks, NaN runs across sub-chunk and super-chunk
    boundaries, series that never see a sample: the fresh-start and carried
    paths of the time-parallel fold against the sequential oracle."""
    rng = np.random.default_rng(17)
    T, S, W = 2400, 200, 60
    X = (500 + 20 * rng.standard_normal((T, S))).astype(np.float32)
    X[:700, :50] = np.nan            # first samples appear mid super-chunk
    X[900:1500, 50:100] = np.nan     # a gap longer than a sub-chunk
    X[:, 100:110] = np.nan           # never a sample
    X[rng.random((T, S)) < 0.2] = np.nan
    ref = native.ewma_z(X, 2 / 61, W)
    for mode in ("1", "2", "3"):
        monkeypatch.setenv("ANOMOD_EWMA_MODE", mode)
        np.testing.assert_allclose(ctx.ewma_z(X, 2 / 61, W), ref, rtol=Z_RTOL, atol=Z_ATOL)


def test_ewma_layout_changes_between_calls(ctx, monkeypatch):
    """A series created for one layout (rows for the time-parallel kernel,
    tiles for the sequential one) and then scored by the other kernel is
    re-laid out on the device; state carries across the switch."""
    rng = np.random.default_rng(5)
    T, S, W = 1000, 150, 50  # T % 16 != 0: a padded last tile
    X = (300 + 5 * rng.standard_normal((2 * T, S))).astype(np.float32)
    X[rng.random((2 * T, S)) < 0.05] = np.nan
    ref = native.ewma_z(X, 0.1, W)
    for first, second in (("2", "1"), ("1", "3"), ("3", "2")):
        monkeypatch.setenv("ANOMOD_EWMA_MODE", first)
        ser = anomod.DeviceSeries(ctx, T, S)
        ser.upload(X[:T])
        z1 = ser.ewma_z(0.1, W)
        monkeypatch.setenv("ANOMOD_EWMA_MODE", second)
        ser.upload(X[T:])
        z2 = ser.ewma_z(0.1, W)
        ser.free()
        np.testing.assert_allclose(np.concatenate([z1, z2]), ref, rtol=Z_RTOL, atol=Z_ATOL)


def test_ewma_synthetic_fill_same_in_both_layouts(ctx, monkeypatch):
    out = []
    for mode in ("1", "3"):
        monkeypatch.setenv("ANOMOD_EWMA_MODE", mode)
        ser = anomod.DeviceSeries(ctx, 1200, 20000)
        ser.fill_synthetic(9, t0=4800)
        out.append(ser.ewma_z(2 / 61, 60))
        ser.free()
    np.testing.assert_array_equal(out[0], out[1])


@pytest.mark.parametrize("mode", ["1", "0"])
def test_ewma_config4_width_matches_oracle(ctx, monkeypatch, mode):
    """BASELINE config 4's width, S = 10^5 series (the bench's tiled layout
    and grid: ANOMOD_EWMA_MODE=1, and whatever auto picks), generated in HBM
    by fill_synthetic (level shifts included), T = 240 steps from t0 = 10^6
    - 120: the z scores equal the C oracle's on the downloaded matrix."""
    monkeypatch.setenv("ANOMOD_EWMA_MODE", mode)
    T, S, W = 240, 100_000, 60
    ser = anomod.DeviceSeries(ctx, T, S)
    ser.fill_synthetic(7, t0=1_000_000 - 120)
    Z = ser.ewma_z(2 / (W + 1), W)
    X = ser.download()
    ser.free()
    assert np.isfinite(X).all()
    np.testing.assert_allclose(Z, native.ewma_z(X, 2 / (W + 1), W), rtol=Z_RTOL, atol=Z_ATOL)


def test_series_download_roundtrip(ctx, ewma_mode):
    rng = np.random.default_rng(4)
    X = rng.standard_normal((100, 333)).astype(np.float32)
    ser = anomod.DeviceSeries(ctx, 100, 333)
    ser.upload(X)
    ser.ewma_z(0.2, 10)  # may re-lay the matrix out for the mode's kernel
    np.testing.assert_array_equal(ser.download(), X)
    ser.free()


def test_ewma_dense_blocks_equal_general_step(ctx, monkeypatch):
    """The tiled kernel takes a select-free step for 64-step blocks in which
    every lane of the wave has started and no sample is NaN.  Waves that are
    wholly dense, that hold one NaN, that start late in one lane, or that hold
    +-inf (sum NaN -> general path; a lone inf stays on the dense path) must
    equal the row kernel (general step only) bit for bit."""
    rng = np.random.default_rng(23)
    T, S, W = 1980, 640, 60  # 10 waves; T % 64 != 0: a partial last block
    X = (1000 + 30 * rng.standard_normal((T, S))).astype(np.float32)
    X[777, 64 + 5] = np.nan                 # wave 1: one NaN in one block
    X[:100, 128 + 9] = np.nan               # wave 2: one lane starts at step 100
    X[1500, 192 + 1] = np.inf               # wave 3: a lone inf (dense path)
    X[300, 256 + 2], X[301, 256 + 3] = np.inf, -np.inf  # wave 4: inf - inf in the sum
    X[:, 320 + 4] = np.nan                  # wave 5: a lane that never starts
    out = []
    for mode in ("1", "3"):
        monkeypatch.setenv("ANOMOD_EWMA_MODE", mode)
        out.append(ctx.ewma_z(X, 2 / 61, W))
    np.testing.assert_array_equal(out[0], out[1])
    fin = np.r_[0:192, 320:640]  # lanes of the waves without inf, against the oracle
    np.testing.assert_allclose(out[0][:, fin], native.ewma_z(X[:, fin], 2 / 61, W),
                               rtol=Z_RTOL, atol=Z_ATOL)


def test_pagerank_matches_networkx_golden(ctx, golden):
    g = np.load(golden / "pagerank_networkx.npz")
    x, it = ctx.pagerank(g["row_ptr"], g["col"], g["w"], g["p"], float(g["alpha"]),
                         iters=1000, tol=1e-12)
    assert it < 1000
    assert np.abs(x - g["x"]).sum() < 1e-5


def test_pagerank_fixed_iters_matches_oracle(ctx):
    rng = np.random.default_rng(4)
    N = 20000
    deg = rng.integers(0, 20, N)
    deg[rng.random(N) < 0.05] = 0
    row_ptr = np.zeros(N + 1, np.uint32)
    np.cumsum(deg, out=row_ptr[1:])
    col = rng.integers(0, N, int(row_ptr[-1])).astype(np.uint32)
    w = rng.integers(1, 1000, col.size).astype(np.float32)
    p = rng.random(N)
    for iters in (1, 2, 37, 100):
        x, it = ctx.pagerank(row_ptr, col, w, p, 0.85, iters=iters, tol=0.0)
        xr, itr = native.pagerank(row_ptr, col, w, p, 0.85, iters=iters, tol=0.0)
        assert it == itr == iters
        assert np.abs(x - xr).sum() < 1e-5


def test_pagerank_config5_graph_matches_oracle(ctx):
    """BASELINE config 5 at size: the synthetic 10^5-node graph the bench
    solves (DeviceGraph(synthetic=...)), 100 fixed iterations and a
    tolerance solve, against the C oracle on the same CSR from the host."""
    g = anomod.DeviceGraph(ctx, synthetic=(100_000, 10, 11))
    rp, col, w = anomod.synth_graph_csr(100_000, 10, 11)
    assert g.nnz == col.shape[0]
    p = np.random.default_rng(0).random(g.N)
    for iters, tol in ((100, 0.0), (1000, 1e-10)):
        x, it = g.pagerank(p, iters=iters, tol=tol)
        xr, itr = native.pagerank(rp, col, w, p, 0.85, iters=iters, tol=tol)
        assert abs(it - itr) <= (0 if tol == 0.0 else 1)  # L1 test: fixed-point vs f64 sums
        assert np.abs(x - xr).sum() < 1e-5
    g.free()


def test_device_graph_replay(ctx):
    g = anomod.DeviceGraph(ctx, synthetic=(100000, 10, 11))
    assert g.N == 100000 and g.nnz > 500000
    p = np.random.default_rng(0).random(g.N)
    x1, _ = g.pagerank(p, iters=100)
    x2, _ = g.pagerank(p, iters=100)
    np.testing.assert_array_equal(x1, x2)
    assert abs(x1.sum() - 1.0) < 1e-6
    g.free()


@pytest.mark.parametrize("sub", ["1", "2", "4"])
def test_pagerank_persistent_equals_per_launch(ctx, monkeypatch, sub):
    """The one-launch solve (grid barrier per iteration; 1, 2 or 4 256-row
    blocks per workgroup) and the per-iteration launches give the same bits
    and stop at the same iteration."""
    g = anomod.DeviceGraph(ctx, synthetic=(100000, 7, 3))
    p = np.random.default_rng(2).random(g.N)
    out = {}
    monkeypatch.setenv("ANOMOD_PPR_SUB", sub)
    for mode in ("2", "1"):  # persistent, per-launch
        monkeypatch.setenv("ANOMOD_PPR_MODE", mode)
        out[mode] = [g.pagerank(p, iters=it, tol=tol) for it, tol in
                     ((1, 0.0), (2, 0.0), (100, 0.0), (1000, 1e-10), (1000, 1e-6))]
    for (xa, ia), (xb, ib) in zip(out["2"], out["1"]):
        assert ia == ib
        np.testing.assert_array_equal(xa, xb)
    assert out["2"][3][1] < 1000 and out["2"][4][1] < out["2"][3][1]
    g.free()


def test_pagerank_persistent_timeout_falls_back(ctx, monkeypatch):
    """A persistent solve whose grid barrier times out (forced: ANOMOD_PPR_SPIN=0,
    no block waits) reruns in-process on the per-launch path and still returns
    the per-launch bits; the path is recorded.  Without the knob the default
    path is the persistent one again."""
    g = anomod.DeviceGraph(ctx, synthetic=(100000, 7, 3))
    p = np.random.default_rng(5).random(g.N)
    cases = ((37, 0.0, "graph"), (1000, 1e-10, "readback"))
    monkeypatch.setenv("ANOMOD_PPR_MODE", "1")
    ref = [g.pagerank(p, iters=it, tol=tol) for it, tol, _ in cases]
    monkeypatch.delenv("ANOMOD_PPR_MODE")
    monkeypatch.setenv("ANOMOD_PPR_SPIN", "0")
    fb0 = g.last_solve()[1]
    for k, ((it, tol, path), (xr, dr)) in enumerate(zip(cases, ref)):
        x, d = g.pagerank(p, iters=it, tol=tol)
        assert g.last_solve() == ("fallback:" + path, fb0 + k + 1)
        assert d == dr
        np.testing.assert_array_equal(x, xr)
    monkeypatch.delenv("ANOMOD_PPR_SPIN")
    x, d = g.pagerank(p, iters=37)
    assert g.last_solve()[0] == "persistent"
    np.testing.assert_array_equal(x, ref[0][0])
    g.free()


@pytest.mark.parametrize("K", [1, 3, 8, 16])
def test_pagerank_batch_equals_single_solves(ctx, K):
    g = anomod.DeviceGraph(ctx, synthetic=(30000, 8, 5))
    rng = np.random.default_rng(K)
    P = rng.random((K, g.N))
    P[:, rng.random(g.N) < 0.5] = 0.0  # sparse personalizations
    for iters, tol in ((37, 0.0), (500, 1e-10)):
        X, done = g.pagerank_batch(P, iters=iters, tol=tol)
        worst = 0
        for k in range(K):
            x, it = g.pagerank(P[k], iters=iters, tol=tol)
            np.testing.assert_array_equal(X[k], x)  # same arithmetic, same order
            worst = max(worst, it)
        assert done == worst
    g.free()


@pytest.mark.parametrize("K,bsub", [(2, None), (5, None), (8, None), (8, "2"), (16, None),
                                    (16, "1")])
def test_pagerank_batch_persistent_equals_per_launch(ctx, monkeypatch, K, bsub):
    """The persistent batch (one launch, grid barrier, vector ring or the
    two-buffer form) == the per-launch batch loop (ANOMOD_PPR_MODE=1), bit
    for bit, in fixed-iteration and tolerance mode (per-vector freezing);
    a barrier timeout (ANOMOD_PPR_SPIN=0) reruns per launch, same bits.
    bsub: 256-row blocks per persistent workgroup (ANOMOD_PPR_BSUB; K = 16
    defaults to 2); K = 16 with the vector ring runs the split kernel (two
    halves of 8 vectors per row), and (16, "1") the one-row-per-lane form
    (ANOMOD_PPR_SPLIT=0)."""
    if bsub:
        monkeypatch.setenv("ANOMOD_PPR_BSUB", bsub)
        if K == 16:
            monkeypatch.setenv("ANOMOD_PPR_SPLIT", "0")
    g = anomod.DeviceGraph(ctx, synthetic=(40000, 9, 12))
    rng = np.random.default_rng(K + 40)
    P = rng.random((K, g.N))
    P[1, rng.random(g.N) < 0.9] = 0.0  # a sparser vector converges at another iteration
    cases = ((1, 0.0), (23, 0.0), (400, 1e-11))
    monkeypatch.setenv("ANOMOD_PPR_MODE", "1")
    ref = [g.pagerank_batch(P, iters=it, tol=tol) for it, tol in cases]
    assert g.last_solve()[0] == "readback"
    monkeypatch.delenv("ANOMOD_PPR_MODE")
    for ring in ("1", "0"):
        monkeypatch.setenv("ANOMOD_PPR_RING", ring)
        for (it, tol), (Xr, dr) in zip(cases, ref):
            X, d = g.pagerank_batch(P, iters=it, tol=tol)
            assert g.last_solve()[0] == "persistent"
            assert d == dr
            np.testing.assert_array_equal(X, Xr)
    monkeypatch.setenv("ANOMOD_PPR_SPIN", "0")
    fb0 = g.last_solve()[1]
    X, d = g.pagerank_batch(P, iters=23)
    assert g.last_solve() == ("fallback:graph", fb0 + 1)
    np.testing.assert_array_equal(X, ref[1][0])
    g.free()


@pytest.mark.parametrize("K", [8, 16])
def test_pagerank_batch_bench_config_is_persistent(ctx, K):
    """The bench's batches (config 5: N = 10^5, 8 and 16 vectors) fit one
    resident grid — K = 8: 391 workgroups of 256 threads, three per CU; K =
    16: 196 workgroups of two 256-row blocks — so each runs as one
    persistent launch, equal to its per-launch solve."""
    g = anomod.DeviceGraph(ctx, synthetic=(100000, 10, 11))
    P = np.random.default_rng(3).random((K, g.N))
    X, d = g.pagerank_batch(P, iters=5)
    assert d == 5 and g.last_solve()[0] == "persistent"
    import os
    os.environ["ANOMOD_PPR_MODE"] = "1"
    try:
        Xr, _ = g.pagerank_batch(P, iters=5)
    finally:
        del os.environ["ANOMOD_PPR_MODE"]
    np.testing.assert_array_equal(X, Xr)
    g.free()


@pytest.mark.parametrize("G", [1, 2, 3, 8, 500])
def test_pagerank_row_sharded_equals_unsharded(ctx, monkeypatch, G):
    """Row-sharded solve rehearsed on one device (G row shards of whole 256-row
    blocks, 500 > blocks: empty shards) == the unsharded per-launch solve, bit
    for bit, in fixed-iteration and tolerance mode."""
    monkeypatch.setenv("ANOMOD_PPR_MODE", "1")
    g = anomod.DeviceGraph(ctx, synthetic=(30000, 8, 6))
    p = np.random.default_rng(G).random(g.N)
    for iters, tol in ((1, 0.0), (37, 0.0), (1000, 1e-10)):
        xs, ds = g.pagerank_sharded(p, iters=iters, tol=tol, virtual_shards=G)
        x, d = g.pagerank(p, iters=iters, tol=tol)
        assert ds == d
        np.testing.assert_array_equal(xs, x)
    x2, _ = g.pagerank(p, iters=37)  # the padded x buffers serve the other paths too
    xs2, _ = g.pagerank_sharded(p, iters=37, virtual_shards=G)
    np.testing.assert_array_equal(x2, xs2)
    g.free()


def test_pagerank_row_sharded_rccl_one_rank(ctx, monkeypatch):
    """The RCCL form (grouped u64 all-reduces + in-place all-gather per
    iteration) on a 1-rank communicator == the unsharded solve."""
    monkeypatch.setenv("ANOMOD_PPR_MODE", "1")
    with anomod.Context(0) as c:
        c.attach_comm(anomod.Context.unique_id(), 1, 0)
        g = anomod.DeviceGraph(c, synthetic=(30000, 8, 6))
        p = np.random.default_rng(1).random(g.N)
        for iters, tol in ((37, 0.0), (1000, 1e-10)):
            xs, ds = g.pagerank_sharded(p, iters=iters, tol=tol)
            x, d = g.pagerank(p, iters=iters, tol=tol)
            assert ds == d
            np.testing.assert_array_equal(xs, x)
        g.free()


def test_features_and_rank_find_injected_fault(ctx):
    fault = "post-storage-service"
    base = anomod.load_experiment(anomod.SynthSpec("SN", seed=21), n_traces=20000)
    exp = anomod.load_experiment(anomod.SynthSpec("SN", seed=22, fault_service=fault),
                                 n_traces=20000)
    fb = anomod.features(base, ctx)
    fe = anomod.features(exp, ctx, baseline=fb)
    assert fe.edges.count.sum() == exp.spans.n_spans
    assert fe.window_scores is not None and fe.window_scores.shape[0] == 480 // 60
    ranking = anomod.rank(fe, ctx=ctx)
    assert anomod.hit_at(ranking, fault, 3) == 1.0


@pytest.mark.parametrize("W", [1, 4, 15])
def test_ewma_on_decoded_prometheus_dir(ctx, golden, ewma_mode, W):
    """§8 row a8 end to end: the SN metric directory the reference wrote
    (tests/golden/prom_dir: NaN gaps, ragged series, +/-inf) -> decoded
    matrix -> EWMA/z kernel == the C oracle on the same matrix."""
    mm = anomod.decode_prometheus_csv_dir(golden / "prom_dir").pad_to_multiple(W)
    assert mm.S == 9 and mm.T >= 30
    a = 2.0 / (W + 1) if W > 1 else 0.3
    np.testing.assert_allclose(ctx.ewma_z(mm.X, a, W), native.ewma_z(mm.X, a, W),
                               rtol=Z_RTOL, atol=Z_ATOL)


@pytest.mark.parametrize("T,S,W,chunk", [(1920, 300, 60, 500), (4800, 77, 16, 1000),
                                         (960, 5000, 96, 100), (1200, 40, 150, 7)])
def test_one_shot_ewma_chunked_equals_one_pass(ctx, ewma_mode, monkeypatch, T, S, W, chunk):
    """anomod_ewma_z streams X through HBM in T-chunks when it exceeds free
    HBM (config 4 on one GPU); ANOMOD_EWMA_CHUNK_STEPS forces the chunking
    here.  Cuts fall on multiples of lcm(16, U), so every kernel's chunked
    scores equal its one-pass scores bit for bit."""
    rng = np.random.default_rng(T * S)
    X = (rng.uniform(0, 1e3, S) + rng.standard_normal((T, S))).astype(np.float32)
    X[rng.random((T, S)) < 0.02] = np.nan
    X[: T // 3, : S // 4] = np.nan  # series that start late, across chunk cuts
    a = 2.0 / (W + 1)
    one = ctx.ewma_z(X, a, W)
    monkeypatch.setenv("ANOMOD_EWMA_CHUNK_STEPS", str(chunk))
    np.testing.assert_array_equal(ctx.ewma_z(X, a, W), one)
    np.testing.assert_allclose(one, native.ewma_z(X, a, W), rtol=Z_RTOL, atol=Z_ATOL)


def test_pagerank_rejects_invalid_personalization(ctx):
    """Negative / NaN / inf entries and an all-zero vector are refused with the
    first bad index (the staging copy is the checking pass); a valid solve
    afterwards gives the same bits as before."""
    g = anomod.DeviceGraph(ctx, synthetic=(5000, 6, 9))
    p = np.random.default_rng(9).random(g.N)
    x0, _ = g.pagerank(p, iters=20)
    for bad_at, v in ((7, -1.0), (4999, np.nan), (0, np.inf), (4093, -np.inf)):
        q = p.copy()
        q[bad_at] = v
        q[bad_at + 1:] = np.where(np.arange(bad_at + 1, g.N) % 2 == 0, -2.0, q[bad_at + 1:])
        with pytest.raises(L.AnomodError, match=rf"personalization\[{bad_at}\] invalid"):
            g.pagerank(q, iters=20)
        with pytest.raises(L.AnomodError, match=rf"personalization\[{bad_at}\] invalid"):
            g.pagerank_sharded(q, iters=20, virtual_shards=2)
        P = np.stack([p, p, q])
        with pytest.raises(L.AnomodError, match=rf"personalization\[2\]\[{bad_at}\] invalid"):
            g.pagerank_batch(P, iters=20)
    with pytest.raises(L.AnomodError, match="sums to zero"):
        g.pagerank(np.zeros(g.N), iters=20)
    x1, _ = g.pagerank(p, iters=20)
    np.testing.assert_array_equal(x0, x1)
    # -0.0 is a valid (zero) weight
    q = p.copy()
    q[3] = -0.0
    g.pagerank(q, iters=5)
    g.free()
