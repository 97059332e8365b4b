"""GPU tests of the host runtime: the C++ train_vae_model loop (mmvae_train) and the drop-in
CLIs bin/nb_vae_main, bin/vmf_vae_main (run on an MI355X: -m gpu).

Chain of checks:
  1. the C++ loop == a Python mirror of mmvae_alg.hh:254-333 driving the same engine through
     the C-ABI (same Philox noise, same bootstrap indices)        -> orchestration is right
  2. the Python mirror with injected noise == the oracle's loop on ATen CPU (the reference's
     op sequence per step)                                        -> loop semantics are right
  3. the CLI on a BGZF MatrixMarket file == the C++ loop on the same data and seed, and writes
     the reference's output files (scores, covariate ones file, recorder tensors).
"""
import gzip
import os
import subprocess

import numpy as np
import pytest
import torch

import mmvae_amd
from helpers import load, golden_files
from mmvae_amd import host
from oracle import nb_oracle, synth, vmf_oracle

pytestmark = pytest.mark.gpu


def kl_beta(epoch, kl_max=1.0, kl_min=0.01, disc=0.1):
    r = np.float32(kl_max) * np.exp(np.float32(-disc) * np.float32(epoch), dtype=np.float32)
    return float(max(np.float32(r), np.float32(kl_min)))


def python_loop(eng, N, B, epochs, nboot, seed, eps_fn=None):
    """mmvae_alg.hh:254-333 over the Python binding (mirror of host/trainer.cc)."""
    nbatch = (N + B - 1) // B
    fwd = 0
    scores = []
    for ep in range(epochs):
        beta = kl_beta(ep)
        tot = np.float32(0)
        for b in range(nbatch):
            batch = (b * B + np.arange(B)) % N
            eps = eps_fn(ep, b, -1) if eps_fn else None
            lb = eng.eval_loss(batch, beta, eps=eps, step_id=fwd, n_total=B)
            fwd += 1
            tot = np.float32(tot + np.float32(lb) * np.float32(B))
            for boot in range(nboot):
                r = host.ridx(seed, ep, b, boot, B)
                eps = eps_fn(ep, b, boot) if eps_fn else None
                eng.step(batch[r], beta, eps=eps, step_id=fwd, n_total=B)
                fwd += 1
        scores.append(float(tot / np.float32(B * nbatch)))
    return np.array(scores, np.float32)


def nb_engine(z, seed=5, dtype="f32", B=None):
    eng = mmvae_amd.Engine(D=int(z["D"]), K=int(z["K"]), max_batch=B or int(z["B"]), dtype=dtype, seed=seed)
    eng.upload_csr(z["rowptr"], z["col"], z["val"])
    eng.init_params(seed=11)
    return eng


def test_cpp_loop_equals_python_mirror():
    z = load(golden_files("nb_mid")[0])
    N, B = int(z["N"]), 64
    a = nb_engine(z, B=B)
    s_cpp = host.train(a, batch_size=B, max_epoch=3, nboot=2, seed=9, recording=1000)
    b = nb_engine(z, B=B)
    s_py = python_loop(b, N, B, 3, 2, 9)
    np.testing.assert_allclose(s_cpp, s_py, rtol=1e-5)
    pa, pb = a.params(registered_only=True), b.params(registered_only=True)
    for k in pa:
        np.testing.assert_allclose(pa[k], pb[k], rtol=1e-4, atol=1e-6, err_msg=k)


def test_python_loop_equals_oracle_loop():
    """Loop semantics vs the reference's: eval forward + nboot resampled Adam steps, scores."""
    z = load(golden_files("nb_small")[0])
    N, D, K, B = int(z["N"]), int(z["D"]), int(z["K"]), 16
    params = {k[5:]: torch.from_numpy(z[k]) for k in z if k.startswith("init/")}
    frozen = {k[7:]: torch.from_numpy(z[k]) for k in z if k.startswith("frozen/")}
    rng = np.random.default_rng(0)
    eps_tab = {}

    def eps_fn(ep, b, boot):
        key = (ep, b, boot)
        if key not in eps_tab:
            eps_tab[key] = (rng.standard_normal((B, K)).astype(np.float32), rng.standard_normal((B, 1)).astype(np.float32))
        m, n = eps_tab[key]
        return np.concatenate([m.ravel(), n.ravel()])

    eng = mmvae_amd.Engine(D=D, K=K, max_batch=B, dtype="f32")
    eng.upload_csr(z["rowptr"], z["col"], z["val"], covar=z["covar"])
    eng.set_params({k: v.numpy() for k, v in params.items()})
    eng.set_params({k: v.numpy() for k, v in frozen.items()})
    s_gpu = python_loop(eng, N, B, 2, 2, 4, eps_fn)
    tr = nb_oracle.NBTrainer(params, frozen)
    nbatch = (N + B - 1) // B
    s_orc = []
    for ep in range(2):
        beta = kl_beta(ep)
        tot = np.float32(0)
        for b in range(nbatch):
            batch = (b * B + np.arange(B)) % N
            x = torch.from_numpy(synth.densify(z["rowptr"], z["col"], z["val"], batch, D))
            c = torch.from_numpy(z["covar"][batch])
            m, n = eps_tab[(ep, b, -1)]
            tot = np.float32(tot + np.float32(tr.eval_loss(x, c, torch.from_numpy(m), torch.from_numpy(n), beta)) * B)
            for boot in range(2):
                r = torch.from_numpy(host.ridx(4, ep, b, boot, B))
                m, n = eps_tab[(ep, b, boot)]
                tr.step(x[r], c[r], torch.from_numpy(m), torch.from_numpy(n), beta)
        s_orc.append(float(tot / np.float32(B * nbatch)))
    np.testing.assert_allclose(s_gpu, s_orc, rtol=2e-4)


def write_bgzf_mtx(path, rowptr, col, val, D):
    from test_host_cpu import bgzf_compress, mtx_text
    with open(path, "wb") as f:
        f.write(bgzf_compress(mtx_text(rowptr, col, val, D)))


def read_gz_matrix(path):
    return np.array([[float(t) for t in ln.split()] for ln in gzip.open(path, "rt").read().splitlines()])


@pytest.mark.parametrize("model", ["nb", "vmf"])
def test_cli_end_to_end(tmp_path, model):
    z = load(golden_files("nb_mid")[0])
    rp, col, val, D, N = z["rowptr"], z["col"], z["val"], int(z["D"]), int(z["N"])
    mtx = str(tmp_path / "data.mtx.gz")
    write_bgzf_mtx(mtx, rp, col, val, D)
    out = str(tmp_path / "run")
    exe = os.path.join(host.BIN_DIR, f"{model}_vae_main")
    lat = ["--mean_latent", "8"] if model == "nb" else ["--latent", "8"]
    r = subprocess.run([exe, "--mtx", mtx, "--out", out, "--batch_size", "64", "--max_epoch", "3", "--nboot", "2",
                        "--recording", "2", "--seed", "3"] + lat, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    scores = np.array([float(s) for s in gzip.open(out + ".scores.gz", "rt").read().split()])
    assert scores.shape == (3,) and np.isfinite(scores).all()
    # the same loop through the library, same data / init / seed
    eng = mmvae_amd.Engine(D=D, K=8, max_batch=64, dtype="f32", seed=3,
                           model=mmvae_amd.MODEL_NB if model == "nb" else mmvae_amd.MODEL_VMF)
    eng.upload_csr(rp, col, val)
    eng.init_params(seed=3)
    s_lib = host.train(eng, batch_size=64, max_epoch=3, nboot=2, seed=3, recording=1000)
    np.testing.assert_allclose(scores, s_lib, rtol=1e-5)
    # outputs of the reference's CLI: the auto covariate file and both column indexes
    # (nb_vae_main.cc:58-59, 68-73)
    assert os.path.exists(out + ".covar.mtx.gz")
    assert host.mtx_read_index(mtx + ".index").size == N
    assert host.mtx_read_index(out + ".covar.mtx.gz.index").size == N
    tag = out + "_1"   # zeropad(epoch 1, max_epoch 3)
    lat_name = ".mu" if model == "nb" else ".latent"
    m = read_gz_matrix(tag + lat_name + "_mean.gz")
    assert m.shape == (N, 8) and np.isfinite(m).all()
    assert read_gz_matrix(tag + lat_name + "_lnvar.gz").shape == (N, 8)
    assert read_gz_matrix(tag + "_x_mean.gz").shape == (1, D)
    assert read_gz_matrix(tag + "_covar_encoding.bias.gz").shape == (8, 1)
    enc = "_mu_encoding.weight.gz" if model == "nb" else "_0.weight.gz"
    assert read_gz_matrix(tag + enc).shape == (8, D)
    # recorder means of the last batch (cells 256..299, 0..19) == the engine's encoder on the
    # parameters at the end of epoch 1 (the recorder encodes each batch after its updates)
    eng2 = mmvae_amd.Engine(D=D, K=8, max_batch=64, dtype="f32", seed=3,
                            model=mmvae_amd.MODEL_NB if model == "nb" else mmvae_amd.MODEL_VMF)
    eng2.upload_csr(rp, col, val)
    eng2.init_params(seed=3)
    host.train(eng2, batch_size=64, max_epoch=2, nboot=2, seed=3, recording=1000)
    em, _ = eng2.encode(np.arange(256, 300))
    np.testing.assert_allclose(m[256:300], em, rtol=2e-3, atol=2e-4)


def test_philox_restatement_matches_engine_noise():
    """oracle/philox.py == the engine's Philox noise (B = 50: no row balancing, staged order =
    batch order), to the device transcendentals' ~1e-6."""
    from oracle import philox
    z = load(golden_files("nb_mid")[0])
    eng = mmvae_amd.Engine(D=int(z["D"]), K=8, max_batch=64, dtype="f32", seed=1234567)
    eng.upload_csr(z["rowptr"], z["col"], z["val"])
    eng.init_params(seed=1)
    eng.eval_loss(np.arange(50), 1.0, step_id=77, row_offset=1000, n_total=5000)
    import ctypes
    got = np.zeros(50 * 8, np.float32)
    assert mmvae_amd.lib().mmvae_debug_copy(eng._h, 3, got.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), got.size) == 0
    got = got.reshape(50, 8)
    want, _ = philox.nb_step_noise(1234567, 77, 50, 8, row_offset=1000)
    np.testing.assert_allclose(got, want, rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("dtype", ["f32", "bf16x3"])
def test_cli_configs0_against_oracle_loop(tmp_path, dtype):
    """BASELINE configs[0]: nb_vae_main on a synthetic 1000 x 500 MatrixMarket file, latent 8,
    batch 100, 3 epochs x 2 bootstrap updates — the CLI's per-epoch scores against the oracle's
    loop (the reference's op sequence on ATen CPU, oracle/nb_oracle.py) from the same initial
    parameters, with the same bootstrap indices and the engine's Philox noise restated in numpy
    (oracle/philox.py)."""
    from oracle import philox
    N, D, K, B, E, NB, SEED = 1000, 500, 8, 100, 3, 2, 5
    rp, col, val = synth.synth_csr(N, D, lib_size=1500.0, seed=21)
    mtx = str(tmp_path / "c0.mtx.gz")
    write_bgzf_mtx(mtx, rp, col, val, D)
    out = str(tmp_path / "run")
    exe = os.path.join(host.BIN_DIR, "nb_vae_main")
    r = subprocess.run([exe, "--mtx", mtx, "--out", out, "--mean_latent", str(K), "--batch_size", str(B),
                        "--max_epoch", str(E), "--nboot", str(NB), "--recording", "1000", "--seed", str(SEED),
                        "--dtype", dtype],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    s_cli = np.array([float(s) for s in gzip.open(out + ".scores.gz", "rt").read().split()])
    # the CLI's initial parameters: mmvae_init_params(seed) on the same cfg
    eng = mmvae_amd.Engine(D=D, K=K, max_batch=B, dtype="f32", seed=SEED)
    eng.upload_csr(rp, col, val)
    eng.init_params(seed=SEED)
    p0 = eng.params()
    shp, fshp = nb_oracle.init_params(D, C=1, K=K)  # the reference's tensor shapes
    params = {k: torch.from_numpy(p0[k].reshape(v.shape).copy()) for k, v in shp.items()}
    frozen = {k: torch.from_numpy(p0[k].reshape(v.shape).copy()) for k, v in fshp.items()}
    tr = nb_oracle.NBTrainer(params, frozen)
    nbatch = (N + B - 1) // B
    fwd, s_orc = 0, []
    for ep in range(E):
        beta = kl_beta(ep)
        tot = np.float32(0)
        for b in range(nbatch):
            batch = (b * B + np.arange(B)) % N
            x = torch.from_numpy(synth.densify(rp, col, val, batch, D))
            c = torch.ones((B, 1), dtype=torch.float32)  # the CLI's automatic ones covariate
            m, n = philox.nb_step_noise(SEED, fwd, B, K)
            fwd += 1
            tot = np.float32(tot + np.float32(tr.eval_loss(x, c, torch.from_numpy(m), torch.from_numpy(n), beta)) * B)
            for boot in range(NB):
                rr = torch.from_numpy(host.ridx(SEED, ep, b, boot, B))
                m, n = philox.nb_step_noise(SEED, fwd, B, K)
                fwd += 1
                tr.step(x[rr], c[rr], torch.from_numpy(m), torch.from_numpy(n), beta)
        s_orc.append(float(tot / np.float32(B * nbatch)))
    np.testing.assert_allclose(s_cli, s_orc, rtol=1e-4)


def test_large_upload_roundtrip_chunked():
    """A CSR above the 32 MB pinned-chunk size (col and val 60 MB each) uploads through the
    double-buffered pinned path and reads back exactly (rows spread over the whole range)."""
    rng = np.random.default_rng(3)
    N, D, per = 30000, 4000, 500
    rp = np.arange(N + 1, dtype=np.int64) * per
    col = np.sort(rng.random((N, D)).argsort(axis=1)[:, :per], axis=1).astype(np.int32).ravel()
    val = rng.integers(1, 50, rp[-1]).astype(np.float32)
    eng = mmvae_amd.Engine(D=D, K=8, max_batch=64, dtype="bf16")
    eng.upload_csr(rp, col, val)
    rows = np.array([0, 1, 777, 15000, 29998, 29999], dtype=np.int64)
    grp, gcol, gval = eng.get_rows(rows)
    want_c = np.concatenate([col[rp[r]:rp[r + 1]] for r in rows])
    want_v = np.concatenate([val[rp[r]:rp[r + 1]] for r in rows])
    np.testing.assert_array_equal(gcol, want_c)
    np.testing.assert_array_equal(gval, want_v)
