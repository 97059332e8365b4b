"""The wide path (mm-vae_amd/csrc/wide.hip) against the oracle (-m gpu).

Shapes the reference trains but the fused tile kernels do not cover — a latent or hidden width
above 64, more than 4 hidden layers, C / H / R above 8, D above 75,264 genes — run on the wide
path: the batch densified into HBM and the reference's op sequence on generic f32-MFMA GEMMs.

* the golden fixtures beyond the fused envelope (nb_wide_*, vmf_wide_*: K = 128, Z = 96,
  --mean_encoding 256,128, six hidden layers, C / H / R = 12 / 10 / 9) report path "wide" and
  follow the oracle's trajectory (they also run through every fixture test of test_gpu_nb.py /
  test_gpu_vmf.py);
* every OTHER golden fixture re-run with the wide path forced (MMVAE_WIDE=1): the two paths are
  held to the same oracle;
* the live oracle at a bench-sized wide shape (NB D = 20k, K = 128, B = 1024) and at D = 80,000
  (above the fused path's gene limit);
* step graphs on the wide path: bit-identical to eager launches, and independent of poisoned
  workspace.
Tolerances: the fp32 ones of the fixture tests (loss 2e-5, gradients 2e-4 norm-relative).
"""
import os

import numpy as np
import pytest
import torch

from helpers import (assert_adam_close, assert_grads_close, engine_from_fixture, eps_of, golden_files, load,
                     params_of, rel_err)

pytestmark = pytest.mark.gpu

WIDE = golden_files("nb_wide") + golden_files("vmf_wide")
FUSED = [p for p in golden_files("nb_") + golden_files("vmf_") if p not in WIDE]


def _eps(z, tag):
    vmf = "model" in z and str(z["model"]) == "vmf"
    return z[f"{tag}/eps_mu"].ravel().astype(np.float32) if vmf else eps_of(z, tag)


def _check_trajectory(z, eng):
    vmf = "model" in z and str(z["model"]) == "vmf"
    prev = params_of(z, "init/")
    for t in range(int(z["steps"])):
        loss, norm = eng.step(z[f"s{t}/cells"], float(z[f"s{t}/beta"]), eps=_eps(z, f"s{t}"))
        want = float(z[f"s{t}/loss"])
        assert abs(loss - want) <= 2e-5 * abs(want), (t, loss, want)
        got, gold = eng.grads(), params_of(z, f"s{t}/grad/")
        if vmf:  # ln_kappa: fp32 cancellation of df/kappa-sized terms (test_gpu_vmf.py)
            gk, wk = float(got.pop("ln_kappa")[0]), float(gold["ln_kappa"][0])
            kap = min(max(float(np.exp(prev["ln_kappa"][0])), 0.1), 10.0)
            df = max(0.5 * int(z["D"]) - 1.0, 0.0)
            assert abs(gk - wk) <= 1e-6 * df / kap + 2e-4 * abs(wk), (t, gk, wk)
        assert_grads_close(got, {k: v for k, v in gold.items() if k in got}, 2e-4, ctx=f"step {t}")
        assert abs(norm - float(z[f"s{t}/total_norm"])) <= 1e-4 * float(z[f"s{t}/total_norm"])
        assert_adam_close(eng.params(registered_only=True), params_of(z, f"s{t}/param/"), gold, ctx=f"step {t}",
                          noisy_keys=("ln_kappa",) if vmf else ())
        prev = params_of(z, f"s{t}/param/")
        eng.set_params(prev)
    steps = int(z["steps"])
    loss = eng.eval_loss(z["eval/cells"], float(z["eval/beta"]), eps=_eps(z, "eval"))
    assert abs(loss - float(z["eval/loss"])) <= 2e-5 * abs(float(z["eval/loss"])), (loss, float(z["eval/loss"]))
    m, lv = eng.encode(z["eval/cells"])
    assert rel_err(m, z["eval/enc_mean"]) < 2e-5
    assert rel_err(lv, z["eval/enc_lnvar"]) < 2e-5
    assert steps >= 2


@pytest.mark.parametrize("path", WIDE, ids=os.path.basename)
def test_wide_fixture_trajectory(path):
    z = load(path)
    eng = engine_from_fixture(z, "bf16x3")
    assert eng.path() == "wide"
    _check_trajectory(z, eng)


@pytest.mark.parametrize("dtype", ["f32", "bf16x3"])
@pytest.mark.parametrize("path", FUSED, ids=os.path.basename)
def test_forced_wide_path_on_every_fixture(monkeypatch, path, dtype):
    """Every fused-shape fixture on the wide path: exact f32 (k_gemm), and bf16x3, which runs the
    MFMA kernels at every fixture's odd shapes — the short-K frozen-weight GEMM (k_gemm_skf) with
    0-2 covariates in its epilogue (3: k_gemm_mf), its column-sum epilogue, ragged row / column tiles."""
    monkeypatch.setenv("MMVAE_WIDE", "1")
    z = load(path)
    eng = engine_from_fixture(z, dtype)
    assert eng.path() == "wide"
    _check_trajectory(z, eng)


def _live(model, D, K, B, N, enc=(), dec=(), C=1, H=1, R=1, relu=False, beta=0.8):
    from mmvae_amd import MODEL_NB, MODEL_VMF, Engine
    from oracle import nb_oracle, synth, vmf_oracle
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    vmf = model == "vmf"
    eng = Engine(D=D, K=K, C=C, H=H, R=R, max_batch=B, dtype="bf16x3", seed=1, relu=relu, enc_hidden=enc,
                 dec_hidden=dec, model=MODEL_VMF if vmf else MODEL_NB)
    assert eng.path() == "wide"
    eng.synth_csr(N, lib_size=2000.0, seed=3)
    eng.init_params(seed=7)
    if vmf:
        eng.set_param("ln_kappa", np.array([np.log(np.float32(4.0))], np.float32))
    cells = (np.arange(B, dtype=np.int64) * 7 + 11) % N
    rng = np.random.default_rng(5)
    em = rng.standard_normal((B, K)).astype(np.float32)
    en = rng.standard_normal((B, R)).astype(np.float32)
    info = {n: k for n, k, _ in eng.param_info()}

    def pull(shapes):
        return {n: torch.from_numpy(eng.get_param(n, info[n]).reshape(v.shape)) for n, v in shapes.items()}
    if vmf:
        p0, f0 = vmf_oracle.init_params(D, C=C, Z=K, enc_layers=enc, dec_layers=dec)
        tr = vmf_oracle.VMFTrainer(pull(p0), pull(f0), relu=relu)
    else:
        p0, f0 = nb_oracle.init_params(D, C=C, K=K, H=H, R=R, enc_layers=enc, dec_layers=dec, relu=relu)
        tr = nb_oracle.NBTrainer(pull(p0), pull(f0), relu=relu)
    eps = em.ravel() if vmf else np.concatenate([em.ravel(), en.ravel()])
    loss, norm = eng.step(cells, beta, eps=eps)
    rp, col, val = eng.get_rows(cells)
    x = torch.from_numpy(synth.densify(rp, col, val, np.arange(B), D))
    c = torch.ones(B, C)
    if vmf:
        r = tr.step(x, c, torch.from_numpy(em), beta)
    else:
        r = tr.step(x, c, torch.from_numpy(em), torch.from_numpy(en), beta)
    assert np.isfinite(loss) and abs(loss - r["loss"]) <= 2e-5 * abs(r["loss"]), (loss, r["loss"])
    gold = {k: v.numpy() for k, v in r["grads"].items()}
    got = eng.grads()
    if vmf:
        gk, wk = float(got.pop("ln_kappa")[0]), float(gold.pop("ln_kappa")[0])
        assert abs(gk - wk) <= 1e-6 * (0.5 * D - 1.0) + 2e-4 * abs(wk), (gk, wk)
    assert_grads_close(got, gold, 2e-4, ctx=f"wide {model} D={D} K={K} B={B}")
    assert abs(norm - r["total_norm"]) <= 2e-3 * r["total_norm"], (norm, r["total_norm"])


def test_wide_nb_latent128_bench_genes():
    """--mean_latent 128 at 20k genes (the reference trains any latent width, nb.hh:59)."""
    _live("nb", 20000, 128, 1024, N=4000)


def test_wide_nb_hidden_256_128():
    """--mean_encoding 256,128 --mean_decoding 128 at 5k genes (nb.hh:331-379)."""
    _live("nb", 5000, 32, 512, N=2000, enc=(256, 128), dec=(128,))


def test_wide_vmf_hidden_relu():
    """vMF --encoding 200,96 --decoding 96 --relu, latent 80 (vmf.hh:338-385)."""
    _live("vmf", 5000, 80, 512, N=2000, enc=(200, 96), dec=(96,), relu=True)


def test_wide_genes_above_fused_limit():
    """D = 80,000 genes: above the batch lists' LDS tile index (75,264), so the wide path."""
    _live("nb", 80000, 16, 128, N=600)


@pytest.mark.parametrize("dtype", ["f32", "bf16x3"])
@pytest.mark.parametrize("model", ["nb", "vmf"])
def test_wide_graph_equals_eager_under_poison(model, dtype):
    """Step graphs on the wide path replay bit-identically to eager launches, with the whole
    workspace (dense blocks, GEMM split partials, latent blocks) poisoned before every step."""
    from mmvae_amd import MODEL_NB, MODEL_VMF, Engine
    D, K, B = 3000, 96, 256
    res = []
    for graph, poison in ((False, None), (True, 0xFF)):
        eng = Engine(D=D, K=K, max_batch=B, dtype=dtype, seed=5, model=MODEL_VMF if model == "vmf" else MODEL_NB)
        assert eng.path() == "wide"
        eng.synth_csr(2000, lib_size=1500.0, seed=4)
        eng.init_params(seed=13)
        eng.graph(graph)
        out = []
        for s, b in enumerate([B, 100, B, 100, 64]):
            if poison is not None:
                eng.poison(poison)
            cells = (np.arange(b, dtype=np.int64) * 3 + 17 * s) % 2000
            out.append(eng.step(cells, 0.6, step_id=s))
        out.append(eng.eval_loss(np.arange(B, dtype=np.int64), 0.6, step_id=9))
        if graph:
            assert eng.graph_stats()["replays"] >= 6
        res.append((out, eng.params(registered_only=True)))
    assert res[0][0] == res[1][0]
    for k in res[0][1]:
        assert np.array_equal(res[0][1][k], res[1][1][k]), k


def test_wide_bf16_operands_latent128():
    """The plain bf16 operand mode on the wide path (k_gemm_mf / k_gemm_skf single-plane
    instances): loss within the bf16 tolerance of the fp32 oracle (2e-3, as the fused bf16 mode)."""
    from mmvae_amd import MODEL_NB, Engine
    from oracle import nb_oracle, synth
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    D, K, B, N = 4000, 128, 512, 1500
    eng = Engine(D=D, K=K, max_batch=B, dtype="bf16", seed=1, model=MODEL_NB)
    assert eng.path() == "wide"
    eng.synth_csr(N, lib_size=2000.0, seed=3)
    eng.init_params(seed=7)
    cells = (np.arange(B, dtype=np.int64) * 7 + 11) % N
    rng = np.random.default_rng(5)
    em = rng.standard_normal((B, K)).astype(np.float32)
    en = rng.standard_normal((B, 1)).astype(np.float32)
    info = {n: k for n, k, _ in eng.param_info()}
    p0, f0 = nb_oracle.init_params(D, C=1, K=K, H=1, R=1)
    pull = {n: torch.from_numpy(eng.get_param(n, info[n]).reshape(v.shape)) for n, v in p0.items()}
    pullf = {n: torch.from_numpy(eng.get_param(n, info[n]).reshape(v.shape)) for n, v in f0.items()}
    tr = nb_oracle.NBTrainer(pull, pullf)
    loss, _ = eng.step(cells, 0.8, eps=np.concatenate([em.ravel(), en.ravel()]))
    rp, col, val = eng.get_rows(cells)
    x = torch.from_numpy(synth.densify(rp, col, val, np.arange(B), D))
    r = tr.step(x, torch.ones(B, 1), torch.from_numpy(em), torch.from_numpy(en), 0.8)
    assert np.isfinite(loss) and abs(loss - r["loss"]) <= 2e-3 * abs(r["loss"]), (loss, r["loss"])
