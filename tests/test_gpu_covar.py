"""One covariate column: the unit-covariate decoder instances against the general ones (-m gpu).

With no covariate file the reference feeds a ones column (nb_vae_main.cc:68-73, vmf_vae_main.cc),
and the engine then runs decoder instances that fold covar_decoding into per-gene constants
(Engine::unit_covar, CM = 0 in nb_kernels.hip / vmf_kernels.hip).  Every C = 1 golden fixture
has that ones column, so these tests pin the other side: a single covariate column that is NOT
all ones must take the general instances and still match the oracle, live, in f32 and x3 — and
a ones column passed explicitly must give the same step as no covariates at all.
"""
import numpy as np
import pytest

from helpers import assert_grads_close, kappa_grad_atol, record_kappa_err

pytestmark = pytest.mark.gpu


def _data(seed, N=300, D=1000):
    from oracle import synth
    rowptr, col, val = synth.synth_csr(N, D, lib_size=400.0, seed=seed)
    cov = (1.0 + 0.5 * np.random.default_rng(seed).standard_normal((N, 1))).astype(np.float32)
    return rowptr, col, val, cov


@pytest.mark.parametrize("dtype", ["f32", "bf16x3"])
def test_nb_single_covariate_column_matches_oracle(dtype):
    from mmvae_amd import Engine
    from oracle import nb_oracle, synth
    import torch
    D, K, B, N = 1000, 16, 200, 300
    rowptr, col, val, cov = _data(31, N, D)
    params, frozen = nb_oracle.init_params(D, K=K, seed=3)
    eng = Engine(D=D, K=K, max_batch=B, dtype=dtype)
    eng.upload_csr(rowptr, col, val, covar=cov)
    eng.set_params({k: v.numpy() for k, v in params.items()})
    eng.set_params({k: v.numpy() for k, v in frozen.items()})
    cells = np.arange(B)
    rng = np.random.default_rng(5)
    em = rng.standard_normal((B, K)).astype(np.float32)
    en = rng.standard_normal((B, 1)).astype(np.float32)
    loss, _ = eng.step(cells, 0.7, eps=np.concatenate([em.ravel(), en.ravel()]))
    tr = nb_oracle.NBTrainer(params, frozen)
    x = torch.from_numpy(synth.densify(rowptr, col, val, cells, D))
    r = tr.step(x, torch.from_numpy(cov[cells]), torch.from_numpy(em), torch.from_numpy(en), 0.7)
    assert abs(loss - r["loss"]) <= 2e-5 * abs(r["loss"])
    assert_grads_close(eng.grads(), {k: v.numpy() for k, v in r["grads"].items()}, 2e-4)


@pytest.mark.parametrize("dtype", ["f32", "bf16x3"])
def test_vmf_single_covariate_column_matches_oracle(dtype):
    from mmvae_amd import MODEL_VMF, Engine
    from oracle import synth, vmf_oracle
    import torch
    D, Z, B, N = 1000, 16, 200, 300
    rowptr, col, val, cov = _data(41, N, D)
    params, frozen = vmf_oracle.init_params(D, Z=Z, seed=3)
    params["ln_kappa"] = torch.tensor([np.log(np.float32(3.0))], dtype=torch.float32)
    eng = Engine(D=D, K=Z, max_batch=B, dtype=dtype, model=MODEL_VMF)
    eng.upload_csr(rowptr, col, val, covar=cov)
    eng.set_params({k: v.numpy() for k, v in params.items()})
    eng.set_params({k: v.numpy() for k, v in frozen.items()})
    cells = np.arange(B)
    eps = np.random.default_rng(5).standard_normal((B, Z)).astype(np.float32)
    loss, _ = eng.step(cells, 0.7, eps=eps.ravel())
    tr = vmf_oracle.VMFTrainer(params, frozen)
    x = torch.from_numpy(synth.densify(rowptr, col, val, cells, D))
    r = tr.step(x, torch.from_numpy(cov[cells]), torch.from_numpy(eps), 0.7)
    assert abs(loss - r["loss"]) <= 2e-5 * abs(r["loss"])
    gold = {k: v.numpy() for k, v in r["grads"].items()}
    gk = gold.pop("ln_kappa")
    got = eng.grads()
    assert_grads_close(got, gold, 2e-4)
    atol = kappa_grad_atol(D, 3.0)  # (ln_kappa = log 3 here; f32 cancellation bound, helpers.py)
    record_kappa_err("covar vmf", D, 3.0, got["ln_kappa"][0], gk[0], atol)
    assert abs(float(got["ln_kappa"][0]) - float(gk[0])) <= atol + 2e-4 * abs(float(gk[0]))


@pytest.mark.parametrize("model", ["nb", "vmf"])
def test_explicit_ones_column_equals_default(model):
    """covar = ones passed explicitly selects the same unit-covariate instances as covar = None:
    bit-identical steps; a column that is ones but for one cell takes the general instances."""
    from mmvae_amd import MODEL_NB, MODEL_VMF, Engine
    D, K, B, N = 1000, 16, 128, 300
    rowptr, col, val, _ = _data(51, N, D)
    ones = np.ones((N, 1), np.float32)
    almost = ones.copy()
    almost[N - 1, 0] = 2.0  # never in the batch below: same data for the batch's rows
    out = []
    for cv in (None, ones, almost):
        eng = Engine(D=D, K=K, max_batch=B, dtype="bf16x3", seed=3, model=MODEL_VMF if model == "vmf" else MODEL_NB)
        eng.upload_csr(rowptr, col, val, covar=cv)
        eng.init_params(seed=9)
        cells = np.arange(B)
        res = [eng.step(cells, 1.0, step_id=s) for s in range(3)]
        out.append((res, eng.params(registered_only=True)))
    assert out[0][0] == out[1][0]
    for k in out[0][1]:
        assert np.array_equal(out[0][1][k], out[1][1][k]), k
    # the general instance: same math up to f32 rounding of the folded constants
    for (la, _), (lb, _) in zip(out[0][0], out[2][0]):
        assert abs(la - lb) <= 2e-5 * abs(la), (la, lb)
