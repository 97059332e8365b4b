"""The per-step batch entry lists' two formats (batch.hip, tiles.hpp EntList; -m gpu).

Integer counts below 2^22 (every scRNA count matrix, and the bench's synthetic data) travel in
the 32-bit entry word itself: bits 0-9 the tile position, bits 10-31 the count.  Any other value
(fractional, negative, -0, >= 2^22) switches the handle's lists to a parallel float array, chosen
at upload from a flag the dataset index kernel sets (resident data) or a host scan (streamed).
MMVAE_LISTS_XM=1 forces the float format.  A count carried either way is the same float, so both
formats must give bit-identical steps; and a dataset with one value past the word's range must
train exactly as the forced float format does."""
import numpy as np
import pytest

from helpers import engine_from_fixture, eps_of, golden_files, load

pytestmark = pytest.mark.gpu


def _csr(N, D, seed, big=None, frac=False):
    rng = np.random.default_rng(seed)
    rows, cols, vals = [], [], []
    rp = [0]
    for c in range(N):
        g = np.sort(rng.choice(D, size=int(rng.integers(0, min(D, 300))), replace=False))
        v = rng.poisson(2.0, size=g.size).astype(np.float32) + 1.0
        if frac and g.size:
            v[0] += 0.25
        cols.append(g.astype(np.int32))
        vals.append(v)
        rp.append(rp[-1] + g.size)
    col = np.concatenate(cols)
    val = np.concatenate(vals)
    if big is not None:
        val[::97] = np.float32(big)  # the largest counts the word carries, or one past it
    return np.asarray(rp, np.int64), col, val


def _run(model, dtype, csr, D, K, B, N, steps=3):
    from mmvae_amd import MODEL_NB, MODEL_VMF, Engine
    eng = Engine(D=D, K=K, max_batch=B, dtype=dtype, model=MODEL_VMF if model == "vmf" else MODEL_NB, seed=3)
    eng.upload_csr(*csr)
    eng.init_params(seed=5)
    out = []
    for t in range(steps):
        cells = (np.arange(B, dtype=np.int64) * (5 + 2 * t) + 3) % N
        out.append(eng.step(cells, 0.7, step_id=t) if t != 1 else (eng.eval_loss(cells, 0.7, step_id=t), 0.0))
    res = (out, eng.grads(), eng.params(registered_only=True))
    eng.close()
    return res


def _same(a, b):
    np.testing.assert_array_equal(np.asarray(a[0]), np.asarray(b[0]))  # (NaN-safe)
    for k in a[1]:
        np.testing.assert_array_equal(a[1][k], b[1][k], err_msg=k)
        np.testing.assert_array_equal(a[2][k], b[2][k], err_msg=k)


@pytest.mark.parametrize("dtype", ["bf16x3", "bf16", "f32"])
@pytest.mark.parametrize("model", ["nb", "vmf"])
def test_count_words_equal_float_lists(monkeypatch, model, dtype):
    """Integer counts: entry-word counts and the forced float lists, bit for bit (ragged B)."""
    D, K, B, N = 3000, 32, 300, 1500
    csr = _csr(N, D, 11)
    monkeypatch.delenv("MMVAE_LISTS_XM", raising=False)
    a = _run(model, dtype, csr, D, K, B, N)
    monkeypatch.setenv("MMVAE_LISTS_XM", "1")
    b = _run(model, dtype, csr, D, K, B, N)
    _same(a, b)


@pytest.mark.parametrize("big,frac", [(4194303.0, False), (4194304.0, False), (None, True)])
def test_values_past_the_word_switch_to_float_lists(monkeypatch, big, frac):
    """2^22 - 1 still fits the word; 2^22 and a fractional value switch the handle to the float
    lists by themselves: each equals the forced float format bit for bit."""
    D, K, B, N = 2000, 32, 256, 1000
    csr = _csr(N, D, 17, big=big, frac=frac)
    monkeypatch.delenv("MMVAE_LISTS_XM", raising=False)
    a = _run("nb", "bf16x3", csr, D, K, B, N, steps=2)
    monkeypatch.setenv("MMVAE_LISTS_XM", "1")
    b = _run("nb", "bf16x3", csr, D, K, B, N, steps=2)
    _same(a, b)


@pytest.mark.parametrize("path", [p for p in golden_files("nb_") if "wide" not in p][:4])
def test_float_lists_meet_the_reference_fixtures(monkeypatch, path):
    """The float-value format against the reference's own fixtures (loss 2e-5, x3)."""
    monkeypatch.setenv("MMVAE_LISTS_XM", "1")
    z = load(path)
    eng = engine_from_fixture(z, "bf16x3")
    loss, _ = eng.step(z["s0/cells"], float(z["s0/beta"]), eps=eps_of(z, "s0"))
    want = float(z["s0/loss"])
    assert abs(loss - want) <= 2e-5 * abs(want), (loss, want)


@pytest.mark.parametrize("model", ["nb", "vmf"])
def test_dense_rows_many_chunks_packed_reads(monkeypatch, model):
    """Rows of several thousand entries (the packed reads' refill of two groups ahead) and 16-row
    blocks past one LDS chunk (~30k entries: several chunks per block): the packed-dataset list
    builder and the unpacked one (MMVAE_LISTS_PK=0) agree bit for bit.  The float-value lists stage
    8 bytes an entry, so their chunks end at other tiles; the raw-count dots riding in the builder
    then sum a row's entries in another lane order, and that format agrees to f32 rounding."""
    from mmvae_amd import MODEL_NB, MODEL_VMF, Engine
    D, K, B, N = 20000, 64 if model == "nb" else 32, 256, 600

    def run():
        eng = Engine(D=D, K=K, max_batch=B, dtype="bf16x3", model=MODEL_VMF if model == "vmf" else MODEL_NB, seed=3)
        nnz = eng.synth_csr(N, lib_size=40000.0, seed=5)
        eng.init_params(seed=5)
        out = []
        for t in range(2):
            cells = (np.arange(B, dtype=np.int64) * (3 + 2 * t) + 1) % N
            out.append(eng.step(cells, 0.7, step_id=t))
        res = (out, eng.grads(), eng.params(registered_only=True))
        eng.close()
        return res, nnz

    for k in ("MMVAE_LISTS_PK", "MMVAE_LISTS_XM"):
        monkeypatch.delenv(k, raising=False)
    a, nnz = run()
    assert nnz / N > 2500, nnz / N  # rows longer than two 1024-entry groups; blocks past one chunk
    monkeypatch.setenv("MMVAE_LISTS_PK", "0")
    b, _ = run()
    monkeypatch.delenv("MMVAE_LISTS_PK")
    monkeypatch.setenv("MMVAE_LISTS_XM", "1")
    c, _ = run()
    _same(a, b)
    from helpers import rel_err
    for (la, na), (lc, nc) in zip(a[0], c[0]):
        assert abs(la - lc) <= 1e-6 * abs(la) and abs(na - nc) <= 1e-5 * abs(na), (la, lc, na, nc)
    for k in a[1]:
        assert rel_err(c[1][k], a[1][k]) <= 1e-5, k


@pytest.mark.parametrize("model", ["nb", "vmf"])
def test_dense_rows_live_oracle(model):
    """The same dense rows (several list chunks per 16-row block) against the live oracle
    (the reference's op sequence): loss 2e-5, gradients 2e-4 in x3."""
    from test_gpu_tiling import _run_live
    _run_live(model, 20000, 64 if model == "nb" else 32, 256, "bf16x3", N=600, lib_size=40000.0, many_tiles=False)


def test_format_switches_on_one_handle(monkeypatch):
    """One handle through resident integer counts (packed copy, count words), the same data streamed
    from host memory, a fractional dataset (float-value lists), and integer counts again: every step
    equals a fresh handle's on the same data bit for bit (the list format, the packed copy and the
    step graphs follow each upload)."""
    from mmvae_amd import MODEL_NB, Engine
    for k in ("MMVAE_LISTS_PK", "MMVAE_LISTS_XM"):
        monkeypatch.delenv(k, raising=False)
    D, K, B, N = 3000, 32, 256, 1200
    ints = _csr(N, D, 23)
    frac = _csr(N, D, 29, frac=True)
    cells = (np.arange(B, dtype=np.int64) * 7 + 2) % N

    def fresh(csr, streamed=False):
        eng = Engine(D=D, K=K, max_batch=B, dtype="bf16x3", model=MODEL_NB, seed=3)
        (eng.stream_csr if streamed else eng.upload_csr)(*csr)
        eng.init_params(seed=5)
        out = eng.step(cells, 0.7, step_id=0), eng.grads()
        eng.close()
        return out

    eng = Engine(D=D, K=K, max_batch=B, dtype="bf16x3", model=MODEL_NB, seed=3)
    eng.graph(True)
    for csr, streamed in ((ints, False), (ints, True), (frac, False), (ints, False)):
        (eng.stream_csr if streamed else eng.upload_csr)(*csr)
        eng.init_params(seed=5)
        eng.reset_optimizer()
        got = eng.step(cells, 0.7, step_id=0), eng.grads()
        want = fresh(csr, streamed)
        assert got[0] == want[0], (streamed, got[0], want[0])
        for k in want[1]:
            np.testing.assert_array_equal(got[1][k], want[1][k], err_msg=f"{k} streamed={streamed}")
    eng.close()
