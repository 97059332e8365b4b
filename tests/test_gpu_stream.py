"""The streamed dataset (mmvae_stream_csr, -m gpu): the CSR stays in host memory and every step
gathers its batch's rows over PCIe into a batch CSR in HBM (csrc/stream.hip) — the reference's
per-batch read of a dataset it never holds whole (mtx_data_block_t::read, mmvae_io.hh:208-245).
The batch's row b is then dataset row b for every kernel after the gather, so a streamed handle
must give bit-identical losses, clip norms, gradients, parameters and encodings to a resident
one (mmvae_upload_csr) on the same data — over ragged batches, bootstrap resampling (duplicate
rows), eval forwards, step graphs, both staging slots, a batch-capacity growth and workspace
poisoning — on the fused NB / vMF kernels and on the wide path.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _data(N, D, seed, C=1):
    from oracle import synth
    rp, col, val = synth.synth_csr(N, D, lib_size=1500.0, seed=seed)
    cov = np.random.default_rng(seed).standard_normal((N, C)).astype(np.float32) if C > 1 else None
    return rp, col, val, cov


def _pair(model, dtype, D, K, B, data, C=1, **kw):
    from mmvae_amd import MODEL_NB, MODEL_VMF, Engine
    rp, col, val, cov = data
    out = []
    for streamed in (False, True):
        eng = Engine(D=D, K=K, C=C, max_batch=B, dtype=dtype, seed=11,
                     model=MODEL_VMF if model == "vmf" else MODEL_NB, **kw)
        if streamed:
            eng.stream_csr(rp, col, val, covar=cov)
        else:
            eng.upload_csr(rp, col, val, covar=cov)
        eng.init_params(seed=5)
        out.append(eng)
    return out


def _drive(eng, N, B, graph, poison):
    eng.graph(graph)
    rng = np.random.default_rng(3)
    res = []
    for s in range(7):
        b = B if s % 3 else B - 37  # ragged every third step
        cells = rng.integers(0, N, b)
        if poison:
            eng.poison(0xFF)
        if s == 2:
            res.append((eng.eval_loss(cells, 0.8, step_id=s), 0.0))
            continue
        ridx = rng.integers(0, b, b) if s == 4 else None  # bootstrap resample: duplicate rows
        res.append(eng.step(cells, 0.8, ridx=ridx, step_id=s))
    m, lv = eng.encode(rng.integers(0, N, B // 2))
    return res, eng.params(registered_only=True), eng.grads(), m, lv


@pytest.mark.parametrize("model,dtype,K", [("nb", "bf16x3", 32), ("nb", "f32", 16), ("nb", "bf16", 64),
                                           ("vmf", "bf16x3", 32), ("nb", "bf16x3", 96), ("vmf", "f32", 80)])
@pytest.mark.parametrize("graph", [False, True])
def test_streamed_equals_resident(model, dtype, K, graph):
    N, D, B = 2500, 3000, 256
    data = _data(N, D, seed=7)
    res, st = _pair(model, dtype, D, K, B, data)
    a = _drive(res, N, B, graph, poison=False)
    b = _drive(st, N, B, graph, poison=graph)  # (poisoned workspace and batch CSR sets)
    assert a[0] == b[0], (a[0], b[0])
    for x, y in ((a[1], b[1]), (a[2], b[2])):
        for k in x:
            assert np.array_equal(x[k], y[k]), k
    assert np.array_equal(a[3], b[3]) and np.array_equal(a[4], b[4])
    if K > 64 or (model == "vmf" and K > 64):
        assert st.path() == "wide"


def test_streamed_covariates_and_rows():
    """Covariates (C = 3) stream with the rows; get_rows reads the caller's arrays."""
    N, D, B = 1200, 2000, 128
    data = _data(N, D, seed=9, C=3)
    res, st = _pair("nb", "bf16x3", D, 16, B, data, C=3)
    rng = np.random.default_rng(1)
    for s in range(3):
        cells = rng.integers(0, N, B)
        assert res.step(cells, 1.0, step_id=s) == st.step(cells, 1.0, step_id=s)
    rows = np.array([0, 7, N - 1, 7], np.int64)
    for x, y in zip(res.get_rows(rows), st.get_rows(rows)):
        assert np.array_equal(x, y)


def test_streamed_batch_growth():
    """A batch heavier than the initial capacity (twice the mean row's share) grows the batch set
    outside the step and re-captures the step graphs; results stay those of the resident handle."""
    from oracle import synth
    N, D, B = 600, 4000, 128
    rp, col, val = synth.synth_csr(N, D, lib_size=800.0, seed=2)
    # 40 heavy cells (lib size 20x), the rest light
    rp2, col2, val2 = synth.synth_csr(40, D, lib_size=16000.0, seed=3)
    rpx = np.concatenate([rp2, rp2[-1] + rp[1:]])
    colx = np.concatenate([col2, col])
    valx = np.concatenate([val2, val])
    res, st = _pair("nb", "bf16x3", D, 32, B, (rpx, colx, valx, None))
    for eng in (res, st):
        eng.graph(True)
    light = np.arange(40, 40 + B, dtype=np.int64)
    heavy = np.arange(0, B, dtype=np.int64) % 40
    for s, cells in enumerate([light, light, heavy, heavy, light]):
        assert res.step(cells, 1.0, step_id=s) == st.step(cells, 1.0, step_id=s), s
    assert st.graph_stats()["captures"] >= 3


@pytest.mark.parametrize("kind", ["fractional", "wide_gene_ids"])
def test_streamed_unpacked_entries(kind):
    """Values that are not 16-bit integer counts (or D > 65536) keep the caller's col / val arrays
    (no packed copy); the steps stay bit-identical to the resident handle."""
    N, B = 800, 128
    D = 3000 if kind == "fractional" else 70000
    rp, col, val, _ = _data(N, D, seed=12)
    if kind == "fractional":
        val = (val * 0.5 + 0.25).astype(np.float32)
    res, st = _pair("nb", "bf16x3", D, 16, B, (rp, col, val, None))
    rng = np.random.default_rng(4)
    for s in range(3):
        cells = rng.integers(0, N, B)
        assert res.step(cells, 1.0, step_id=s) == st.step(cells, 1.0, step_id=s), s


@pytest.mark.parametrize("mode", [("MMVAE_STREAM_DMA", "0"), ("MMVAE_STREAM_THP", "1"), ("MMVAE_STREAM_INDEX_STEP", "1"),
                                  ("MMVAE_STREAM_SYNC", "1"), ("MMVAE_STREAM_B3", "1")])
def test_streamed_modes(mode, monkeypatch):
    """The streamed path's alternative modes (read at stream_csr): the zero-copy gather kernel
    (no DMA copy), its huge-page packed copy, the batch index built inside the step, the in-step
    gather — each bit-identical to the resident handle over ragged, resampled and eval steps
    with step graphs and workspace poisoning."""
    monkeypatch.setenv(*mode)
    if mode[0] in ("MMVAE_STREAM_THP", "MMVAE_STREAM_INDEX_STEP"):
        monkeypatch.setenv("MMVAE_STREAM_DMA", "0")  # (zero-copy gather options)
    N, D, B = 1500, 3000, 192
    data = _data(N, D, seed=21)
    res, st = _pair("nb", "bf16x3", D, 32, B, data)
    a = _drive(res, N, B, True, poison=False)
    b = _drive(st, N, B, True, poison=True)
    assert a[0] == b[0], (a[0], b[0])
    for x, y in ((a[1], b[1]), (a[2], b[2])):
        for k in x:
            assert np.array_equal(x[k], y[k]), k
    assert np.array_equal(a[3], b[3]) and np.array_equal(a[4], b[4])


@pytest.mark.parametrize("b3", ["0", "1"])
def test_streamed_dma_buffer_growth(b3, monkeypatch):
    """The DMA mode's slot buffers grow on their own (a batch 1.25x heavier than the first one)
    while the batch sets do not: the step graphs that read the old buffer are re-captured (4-byte
    and 3-byte entries)."""
    monkeypatch.setenv("MMVAE_STREAM_B3", b3)
    from oracle import synth
    N, D, B = 1200, 3000, 128
    rp, col, val = synth.synth_csr(N // 2, D, lib_size=600.0, seed=5)
    rp2, col2, val2 = synth.synth_csr(N // 2, D, lib_size=1800.0, seed=6)
    rpx = np.concatenate([rp, rp[-1] + rp2[1:]])
    colx = np.concatenate([col, col2])
    valx = np.concatenate([val, val2])
    res, st = _pair("nb", "bf16x3", D, 32, B, (rpx, colx, valx, None))
    for eng in (res, st):
        eng.graph(True)
    light = np.arange(0, B, dtype=np.int64)
    heavy = np.arange(N // 2, N // 2 + B, dtype=np.int64)
    for s, cells in enumerate([light, light, light, heavy, heavy, light, heavy]):
        assert res.step(cells, 1.0, step_id=s) == st.step(cells, 1.0, step_id=s), s
    for k, v in res.params(registered_only=True).items():
        assert np.array_equal(v, st.params(registered_only=True)[k]), k


@pytest.mark.parametrize("mode", [None, ("MMVAE_STREAM_DMA", "0")])
def test_streamed_async_pipeline(mode, monkeypatch):
    """the host runs ahead (run(sync=False)): both staging slots and both batch sets are in
    flight while the prefetched gather (DMA copy or zero-copy kernel) of step n + 1 overlaps step n —
    the ordering that ev_setfree, ev_gathered and the staging tickets carry — including steps whose
    heavier batch grows the batch sets / DMA buffers mid-stream.  Parameters and gradients after the
    run, and the closing synced step's loss, must equal the resident handle's bit for bit."""
    if mode:
        monkeypatch.setenv(*mode)
    from oracle import synth
    N, D, B = 1200, 3000, 128
    rp, col, val = synth.synth_csr(N // 2, D, lib_size=600.0, seed=15)
    rp2, col2, val2 = synth.synth_csr(N // 2, D, lib_size=2400.0, seed=16)
    data = (np.concatenate([rp, rp[-1] + rp2[1:]]), np.concatenate([col, col2]), np.concatenate([val, val2]), None)
    res, st = _pair("nb", "bf16x3", D, 32, B, data)
    rng = np.random.default_rng(8)
    plan = []
    for s in range(12):
        heavy = s in (4, 5, 9)
        b = B - 21 if s == 7 else B
        cells = rng.integers(N // 2, N, b) if heavy else rng.integers(0, N // 2, b)
        plan.append((cells, s == 6, rng.integers(0, b, b) if s == 8 else None))
    for eng in (res, st):
        eng.graph(True)
        for s, (cells, ev, ridx) in enumerate(plan):
            eng.run(cells, 0.9, ridx=ridx, update=not ev, step_id=s, sync=False)
        eng.sync()
    for x, y in ((res.params(registered_only=True), st.params(registered_only=True)), (res.grads(), st.grads())):
        for k in x:
            assert np.array_equal(x[k], y[k]), k
    cells = rng.integers(0, N, B)
    assert res.step(cells, 0.9, step_id=99) == st.step(cells, 0.9, step_id=99)


@pytest.mark.parametrize("kind", ["packed", "unpacked"])
def test_released_stream_arrays_reused_by_a_resident_upload(kind):
    """The round-5 fault's sequence, made deterministic.  Until 3a24d7a the streamed
    handle page-locked the caller's own arrays (hipHostRegister) and unregistered them at release.
    In the suite, a streamed test's arrays were freed while its handle was still alive (the handle
    went later, with the garbage collector); the next test allocated same-size arrays at the same
    addresses, and its resident upload's plain host-to-device copy of `col` faulted ("illegal
    memory access" in upload_chunked(d_col)).  Here: a streamed handle takes arrays A; A is freed
    while the handle lives; new arrays A' are allocated (same sizes, typically the same addresses)
    and a resident handle uploads from A' and trains; the streamed handle is then destroyed and a
    second resident handle uploads from A' again.  Every result must equal a clean handle's, bit
    for bit, with the streamed handle stepping in between (it must still read its own copies)."""
    import gc
    from mmvae_amd import MODEL_NB, Engine
    N, D, B, K = 2500, 3000 if kind == "packed" else 70000, 256, 32
    rp0, col0, val0, _ = _data(N, min(D, 3000), seed=21)
    if kind == "unpacked":
        val0 = val0 + np.float32(0.25)  # fractional values: the unpacked col / val pinned copies

    def fresh():
        return rp0.copy(), col0.copy(), val0.copy()

    def run(eng):
        eng.init_params(seed=5)
        rng = np.random.default_rng(8)
        return [eng.step(rng.integers(0, N, B), 0.8, step_id=s) for s in range(3)], eng.params(registered_only=True)

    def make():
        return Engine(D=D, K=K, max_batch=B, dtype="bf16x3", seed=11, model=MODEL_NB)

    clean = make()
    clean.upload_csr(*fresh())
    want, want_p = run(clean)
    clean.close()

    a = fresh()
    old_addr = [x.ctypes.data for x in a]
    streamed = make()
    streamed.stream_csr(*a)
    s_res = run(streamed)
    del a
    gc.collect()
    a2 = fresh()  # same sizes: the allocator hands back the freed ranges as a rule
    reused = sum(x.ctypes.data == o for x, o in zip(a2, old_addr))
    r1 = make()
    r1.upload_csr(*a2)
    got1, got1_p = run(r1)
    # the streamed handle still reads its own (engine-owned) copies of the freed arrays
    s_again = run(streamed)
    streamed.close()
    r1.close()
    r2 = make()
    r2.upload_csr(*a2)
    got2, got2_p = run(r2)
    r2.close()
    assert got1 == want and got2 == want, (reused, got1, got2, want)
    assert s_res[0] == want and s_again[0] == want, (s_res[0], s_again[0], want)
    for k in want_p:
        assert np.array_equal(got1_p[k], want_p[k]) and np.array_equal(got2_p[k], want_p[k]), k
