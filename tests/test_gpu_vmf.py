"""GPU parity tests of the vMF ELBO step through the C-ABI (run on an MI355X: -m gpu).

libmmvae.so's vMF kernels (mm-vae_amd/csrc/vmf_kernels.hip) against the oracle's golden
vectors (tests/golden/vmf_*.npz, oracle/vmf_oracle.py = vmf.hh:250-440 on ATen fp32) and
size-independent properties at the bench size.
Tolerances: fp32 mode loss rel <= 2e-5, gradients norm-relative <= 2e-4 per tensor, except
ln_kappa: its gradient is df/kappa - (B/n) df/kappa-scale cancellation (the lbessel backward
returns the Baricz bound ~ df/kappa, Q3) so it carries fp32 noise of a few ulp of df/kappa in
the reference itself: absolute tolerance 8 ulp_f32(df / kappa) * kappa (helpers.kappa_grad_atol,
derived there), every measured difference logged to gpurun_out/kappa_grad_err.jsonl.  bf16 mode:
loss rel <= 2e-3, gradients norm-relative <= 3e-2.
"""
import os

import numpy as np
import pytest

from helpers import (assert_adam_close, assert_grads_close, dims, engine_from_fixture, golden_files,
                     kappa_grad_atol, load, params_of, record_kappa_err, rel_err)

pytestmark = pytest.mark.gpu
VMF_FILES = golden_files("vmf_")


def eps_v(z, tag):
    return z[f"{tag}/eps_mu"].ravel().astype(np.float32)


def kappa_atol(z, params):
    kap = min(max(float(np.exp(params["ln_kappa"][0])), 0.1), 10.0)
    return kappa_grad_atol(int(z["D"]), kap)


def check_grads(got, gold, tol, atol_k, ctx, D=0, kappa=0.0):
    g = dict(gold)
    gk = g.pop("ln_kappa")
    assert_grads_close(got, g, tol, ctx=ctx)
    if D:
        record_kappa_err(ctx, D, kappa, got["ln_kappa"][0], gk[0], atol_k)
    assert abs(float(got["ln_kappa"][0]) - float(gk[0])) <= atol_k + tol * abs(float(gk[0])), \
        (ctx, float(got["ln_kappa"][0]), float(gk[0]))


@pytest.mark.parametrize("dtype", ["f32", "bf16x3"])
@pytest.mark.parametrize("path", VMF_FILES, ids=os.path.basename)
def test_vmf_fp32_parity_trajectory(path, dtype):
    z = load(path)
    eng = engine_from_fixture(z, dtype)
    prev = params_of(z, "init/")
    for t in range(int(z["steps"])):
        loss, norm = eng.step(z[f"s{t}/cells"], float(z[f"s{t}/beta"]), eps=eps_v(z, f"s{t}"))
        want = float(z[f"s{t}/loss"])
        assert abs(loss - want) <= 2e-5 * abs(want), (t, loss, want)
        gold = params_of(z, f"s{t}/grad/")
        check_grads(eng.grads(), gold, 2e-4, kappa_atol(z, prev), f"{os.path.basename(path)} {dtype} step {t}",
                    D=int(z["D"]), kappa=min(max(float(np.exp(prev["ln_kappa"][0])), 0.1), 10.0))
        assert abs(norm - float(z[f"s{t}/total_norm"])) <= 1e-4 * float(z[f"s{t}/total_norm"])
        assert_adam_close(eng.params(registered_only=True), params_of(z, f"s{t}/param/"), gold, ctx=f"step {t}",
                          noisy_keys=("ln_kappa",))
        prev = params_of(z, f"s{t}/param/")
        eng.set_params(prev)


@pytest.mark.parametrize("dtype", ["f32", "bf16x3"])
@pytest.mark.parametrize("path", VMF_FILES, ids=os.path.basename)
def test_vmf_eval_and_encode(path, dtype):
    z = load(path)
    eng = engine_from_fixture(z, dtype)
    steps = int(z["steps"])
    eng.set_params(params_of(z, f"s{steps - 1}/param/"))
    loss = eng.eval_loss(z["eval/cells"], float(z["eval/beta"]), eps=eps_v(z, "eval"))
    assert abs(loss - float(z["eval/loss"])) <= 2e-5 * abs(float(z["eval/loss"]))
    m, lv = eng.encode(z["eval/cells"])
    assert rel_err(m, z["eval/enc_mean"]) < 2e-5
    assert rel_err(lv, z["eval/enc_lnvar"]) < 2e-5


@pytest.mark.parametrize("path", VMF_FILES, ids=os.path.basename)
def test_vmf_bf16_close(path):
    z = load(path)
    eng = engine_from_fixture(z, "bf16")
    loss, _ = eng.step(z["s0/cells"], float(z["s0/beta"]), eps=eps_v(z, "s0"))
    want = float(z["s0/loss"])
    assert abs(loss - want) <= 2e-3 * abs(want)
    g = params_of(z, "s0/grad/")
    check_grads(eng.grads(), g, 3e-2, 3e-2 * max(abs(float(g["ln_kappa"][0])), 1.0), "bf16")


def test_vmf_ragged_and_empty_rows():
    """B not a multiple of 64, empty cells (y = uniform 1/sqrt(D)), genes past the last full tile."""
    import torch
    from mmvae_amd import MODEL_VMF, Engine
    from oracle import synth, vmf_oracle
    D, Z, B, N = 1000, 16, 200, 300
    rowptr, col, val = synth.synth_csr(N, D, lib_size=400.0, seed=21)
    for r in (5, 17):
        n = rowptr[r + 1] - rowptr[r]
        col = np.delete(col, np.s_[rowptr[r]:rowptr[r + 1]])
        val = np.delete(val, np.s_[rowptr[r]:rowptr[r + 1]])
        rowptr[r + 1:] -= n
    params, frozen = vmf_oracle.init_params(D, Z=Z, seed=3)
    params["ln_kappa"] = torch.tensor([np.log(np.float32(3.0))], dtype=torch.float32)
    eng = Engine(D=D, K=Z, max_batch=B, dtype="f32", model=MODEL_VMF)
    eng.upload_csr(rowptr, col, val)
    eng.set_params({k: v.numpy() for k, v in params.items()})
    eng.set_params({k: v.numpy() for k, v in frozen.items()})
    cells = np.arange(B)
    eps = np.random.default_rng(5).standard_normal((B, Z)).astype(np.float32)
    loss, _ = eng.step(cells, 0.7, eps=eps.ravel())
    tr = vmf_oracle.VMFTrainer(params, frozen)
    x = torch.from_numpy(synth.densify(rowptr, col, val, cells, D))
    r = tr.step(x, torch.ones(B, 1), torch.from_numpy(eps), 0.7)
    assert abs(loss - r["loss"]) <= 2e-5 * abs(r["loss"])
    gold = {k: v.numpy() for k, v in r["grads"].items()}
    check_grads(eng.grads(), gold, 2e-4, kappa_grad_atol(D, 3.0), "ragged", D=D, kappa=3.0)


def test_vmf_philox_noise_world_invariant():
    z = load([p for p in VMF_FILES if p.endswith("vmf_k32.npz")][0])
    d = dims(z)
    cells = z["s0/cells"]
    full = engine_from_fixture(z, "f32")
    l_full = full.eval_loss(cells, 1.0, step_id=3)
    half = d["B"] // 2
    parts = []
    for r in range(2):
        eng = engine_from_fixture(z, "f32")
        parts.append(eng.eval_loss(cells[r * half:(r + 1) * half], 1.0, n_total=d["B"], row_offset=r * half,
                                   step_id=3))
    assert abs(sum(parts) - l_full) <= 1e-5 * abs(l_full)


def test_vmf_full_size_properties():
    """D = 20k, Z = 32, B = 4096 (BASELINE config 3): finite, deterministic, loss decreases,
    fp32 and bf16 agree."""
    from mmvae_amd import MODEL_VMF, Engine
    D, Z, B = 20000, 32, 4096
    losses = {}
    for dt in ("bf16", "f32"):
        eng = Engine(D=D, K=Z, max_batch=B, dtype=dt, seed=1, model=MODEL_VMF)
        eng.synth_csr(20000, lib_size=2000.0, seed=3)
        eng.init_params(seed=7)
        cells = np.arange(B)
        l0 = eng.eval_loss(cells, 1.0, step_id=0)
        l0b = eng.eval_loss(cells, 1.0, step_id=0)
        assert abs(l0 - l0b) <= 1e-6 * abs(l0) and np.isfinite(l0)
        ls = [eng.step(cells, 1.0, step_id=i)[0] for i in range(6)]
        assert all(np.isfinite(ls)) and ls[-1] < ls[0], ls
        losses[dt] = l0
        assert all(np.isfinite(v).all() for v in eng.grads().values())
    assert abs(losses["bf16"] - losses["f32"]) <= 2e-3 * abs(losses["f32"])


def test_vmf_split_gradient_buckets_agree(monkeypatch):
    """Data-parallel vMF step: covar_decoding_ gradients finalised right after k_vdec_bwd (their
    all-reduce overlaps the encoder backward), x_mean / ln_x_sd at the end (MMVAE_SPLIT_GRADS=1
    forces that path at world size 1) — bit-identical to the single finalisation."""
    import mmvae_amd
    D, K, B, N = 3000, 32, 512, 2000
    out = {}
    for split in ("0", "1"):
        monkeypatch.setenv("MMVAE_SPLIT_GRADS", split)
        eng = mmvae_amd.Engine(D=D, K=K, max_batch=B, dtype="bf16", seed=1, model=mmvae_amd.MODEL_VMF)
        eng.synth_csr(N, lib_size=2000.0, seed=5)
        eng.init_params(seed=11)
        res = [eng.step(np.arange(B) * 3 % N, 0.5, step_id=t) for t in range(2)]
        out[split] = (res, eng.grads(), eng.params(registered_only=True))
    (r0, g0, p0), (r1, g1, p1) = out["0"], out["1"]
    assert r0 == r1
    for k in g0:
        np.testing.assert_array_equal(g0[k], g1[k], err_msg=k)
        np.testing.assert_array_equal(p0[k], p1[k], err_msg=k)
