"""CPU tests of the vMF oracle and of the kernel algebra the vMF HIP path implements.

* the oracle (oracle/vmf_oracle.py = vmf.hh:250-440 op sequence on ATen fp32) reproduces
  every committed vMF golden fixture bit for bit;
* oracle/vmf_analytic.py (the float64 restatement of vmf_kernels.hip's algebra) equals
  LibTorch autograd of the oracle run in float64, and the fp32 golden gradients.
"""
import os

import numpy as np
import pytest
import torch

from helpers import dims, golden_files, load, params_of, relu_of
from oracle import synth, vmf_analytic, vmf_oracle

VMF_FILES = golden_files("vmf_")


def test_vmf_golden_fixtures_present():
    assert len(VMF_FILES) >= 5


@pytest.mark.parametrize("path", VMF_FILES, ids=os.path.basename)
def test_vmf_oracle_reproduces_golden(path):
    z = load(path)
    d = dims(z)
    torch.set_num_threads(1)
    tr = vmf_oracle.VMFTrainer({k: torch.from_numpy(v) for k, v in params_of(z, "init/").items()},
                               {k: torch.from_numpy(v) for k, v in params_of(z, "frozen/").items()}, relu=relu_of(z))
    for t in range(int(z["steps"])):
        cells = z[f"s{t}/cells"]
        x = torch.from_numpy(synth.densify(z["rowptr"], z["col"], z["val"], cells, d["D"]))
        c = torch.from_numpy(z["covar"][cells])
        r = tr.step(x, c, torch.from_numpy(z[f"s{t}/eps_mu"]), float(z[f"s{t}/beta"]))
        assert np.float32(r["loss"]) == z[f"s{t}/loss"]
        for k, v in r["grads"].items():
            np.testing.assert_array_equal(v.numpy(), z[f"s{t}/grad/{k}"])
        for k, v in tr.params().items():
            np.testing.assert_array_equal(v.numpy(), z[f"s{t}/param/{k}"])


@pytest.mark.parametrize("path", VMF_FILES, ids=os.path.basename)
def test_vmf_kernel_algebra_equals_autograd_f64(path):
    z = load(path)
    d = dims(z)
    P = {k: torch.from_numpy(v.astype(np.float64)) for k, v in params_of(z, "s0/param/").items()}
    FR = {k: torch.from_numpy(v.astype(np.float64)) for k, v in params_of(z, "frozen/").items()}
    cells = z["s1/cells"]
    x = torch.from_numpy(synth.densify(z["rowptr"], z["col"], z["val"], cells, d["D"]).astype(np.float64))
    c = torch.from_numpy(z["covar"][cells].astype(np.float64))
    eps = torch.from_numpy(z["s1/eps_mu"].astype(np.float64))
    beta = float(z["s1/beta"])
    m = vmf_oracle.VMFModel(P, FR, relu=relu_of(z))
    L = vmf_oracle.vmf_vae_loss(x, m.forward(x, c, eps, True), beta)
    L.backward()
    La, G = vmf_analytic.vmf_step_grads({k: v.numpy() for k, v in P.items()}, {k: v.numpy() for k, v in FR.items()},
                                        x.numpy(), c.numpy(), eps.numpy(), beta, relu=relu_of(z))
    assert abs(La - float(L.detach())) <= 1e-7 * abs(La)
    for k, t in m.p.items():
        g = t.grad.numpy().ravel()
        a = np.asarray(G[k]).ravel()
        assert np.abs(g - a).max() <= 1e-9 * (np.abs(g).max() + 1e-12) + 1e-12, k


@pytest.mark.parametrize("path", VMF_FILES, ids=os.path.basename)
def test_vmf_kernel_algebra_matches_golden_fp32(path):
    z = load(path)
    d = dims(z)
    P = {k: v.astype(np.float64) for k, v in params_of(z, "init/").items()}
    FR = {k: v.astype(np.float64) for k, v in params_of(z, "frozen/").items()}
    cells = z["s0/cells"]
    x = synth.densify(z["rowptr"], z["col"], z["val"], cells, d["D"]).astype(np.float64)
    L, G = vmf_analytic.vmf_step_grads(P, FR, x, z["covar"][cells].astype(np.float64),
                                       z["s0/eps_mu"].astype(np.float64), float(z["s0/beta"]), relu=relu_of(z))
    assert abs(L - float(z["s0/loss"])) <= 1e-5 * abs(L)
    for k in vmf_oracle.param_names():
        want = z[f"s0/grad/{k}"].astype(np.float64).ravel()
        got = np.asarray(G[k], np.float64).ravel()
        assert np.abs(got - want).max() <= 2e-4 * np.abs(got).max() + 1e-7, k


def test_vmf_kappa_init_mask_q4():
    """ln_kappa = log(kappa_min) in fp32 gives exp() just below kappa_min: the clamp passes
    no gradient at the first step; vmf_small starts there."""
    z = load([p for p in VMF_FILES if p.endswith("vmf_small.npz")][0])
    assert float(z["s0/grad/ln_kappa"][0]) == 0.0
    assert float(z["s1/grad/ln_kappa"][0]) != 0.0
