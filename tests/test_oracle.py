"""CPU tests: the oracle against the golden vectors and against the reference itself.

* fast-math helpers vs the reference's own fastlog.h/fastgamma.h (oracle/_ref, built from
  /root/reference when present) — bit-exact;
* every NB golden fixture is an output of the reference's own nb.hh model + Adam loop
  (oracle/ref_nb_harness.cc); where the harness is built, it is re-run on each fixture's
  inputs and must reproduce the fixture bit for bit (parity pinned to the reference);
* the oracle reproduces every NB golden fixture — i.e. the reference's numbers — bit for bit;
* the float64 restatement of the kernel algebra (oracle/nb_analytic.py) equals the
  oracle's LibTorch-autograd loss and gradients.
"""
import ctypes
import os

import numpy as np
import pytest
import torch

from helpers import GOLDEN, dims, golden_files, load, params_of, relu_of
from oracle import fastmath, nb_analytic, nb_oracle, ref_nb, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref_fastmath.so")


@pytest.mark.skipif(not os.path.exists(REF_SO), reason="oracle/_ref not built (needs /root/reference)")
def test_fastmath_bit_exact_vs_reference():
    L = ctypes.CDLL(REF_SO)
    for fn in ("ref_fasterlog", "ref_fasterlgamma"):
        getattr(L, fn).restype = ctypes.c_float
        getattr(L, fn).argtypes = [ctypes.c_float]
    xs = np.concatenate([np.float32([2 * np.pi, 25.0, 10001.0, 1.0, 0.5]),
                         np.random.default_rng(0).uniform(1e-3, 3e4, 2000).astype(np.float32)])
    for x in xs:
        assert np.float32(L.ref_fasterlog(x)).tobytes() == np.float32(fastmath.fasterlog(x)).tobytes()
        assert np.float32(L.ref_fasterlgamma(x)).tobytes() == np.float32(fastmath.fasterlgamma(x)).tobytes()


def test_fastmath_known_constants():
    # fasterlog(2 pi) = 1.82167053, fasterlgamma(25) = 54.4777
    assert abs(float(fastmath.fasterlog(np.float32(2 * np.pi))) - 1.82167053) < 1e-6
    assert abs(float(fastmath.fasterlgamma(np.float32(25.0))) - 54.4777) < 1e-3


def test_nb_fixtures_come_from_the_reference():
    for p in golden_files("nb_"):
        assert str(load(p)["source"]).startswith("reference nb.hh:1-563"), p


@pytest.mark.skipif(not ref_nb.available(), reason="oracle/_ref/ref_nb_harness not built (needs /root/reference)")
@pytest.mark.parametrize("path", golden_files("nb_"), ids=os.path.basename)
def test_reference_reproduces_golden(path):
    """Re-run the reference (nb.hh:1-563, mmvae_alg.hh:234-310 on LibTorch) on the fixture's
    parameters, rows and seeds: every stored number must come back bit for bit."""
    z = load(path)
    d = dims(z)
    enc, dec = (tuple(int(v) for v in z[k]) for k in ("enc_layers", "dec_layers"))
    params = {**params_of(z, "init/"), **params_of(z, "frozen/")}
    def rows(cells):
        return synth.densify(z["rowptr"], z["col"], z["val"], cells, d["D"]), z["covar"][cells]
    sched = []
    for t in range(int(z["steps"])):
        x, c = rows(z[f"s{t}/cells"])
        sched.append(dict(x=x, c=c, ridx=np.arange(d["B"]), beta=float(z[f"s{t}/beta"]),
                          seed=int(z[f"s{t}/torch_seed"])))
    x, c = rows(z["eval/cells"])
    evalb = dict(x=x, c=c, beta=float(z["eval/beta"]), seed=int(z["eval/torch_seed"]))
    ref = ref_nb.run(d["D"], d["C"], d["K"], d["H"], d["R"], relu_of(z), 0, enc, dec, sched, evalb,
                     params_in={k.replace("frozen/", ""): v for k, v in params.items()})
    for k, v in ref.items():
        np.testing.assert_array_equal(np.asarray(v, z[k].dtype).reshape(z[k].shape), z[k], err_msg=k)


@pytest.mark.parametrize("path", golden_files("nb_"), ids=os.path.basename)
def test_oracle_reproduces_golden(path):
    z = load(path)
    d = dims(z)
    torch.set_num_threads(1)
    tr = nb_oracle.NBTrainer({k: torch.from_numpy(v) for k, v in params_of(z, "init/").items()},
                             {k: torch.from_numpy(v) for k, v in params_of(z, "frozen/").items()}, relu=relu_of(z))
    for t in range(int(z["steps"])):
        cells = z[f"s{t}/cells"]
        x = torch.from_numpy(synth.densify(z["rowptr"], z["col"], z["val"], cells, d["D"]))
        c = torch.from_numpy(z["covar"][cells])
        r = tr.step(x, c, torch.from_numpy(z[f"s{t}/eps_mu"]), torch.from_numpy(z[f"s{t}/eps_nu"]),
                    float(z[f"s{t}/beta"]))
        assert np.float32(r["loss"]) == z[f"s{t}/loss"]
        for k, v in r["grads"].items():
            np.testing.assert_array_equal(v.numpy(), z[f"s{t}/grad/{k}"])
        for k, v in tr.params().items():
            np.testing.assert_array_equal(v.numpy(), z[f"s{t}/param/{k}"])
    cells = z["eval/cells"]
    x = torch.from_numpy(synth.densify(z["rowptr"], z["col"], z["val"], cells, d["D"]))
    el = tr.eval_loss(x, torch.from_numpy(z["covar"][cells]), torch.from_numpy(z["eval/eps_mu"]),
                      torch.from_numpy(z["eval/eps_nu"]), float(z["eval/beta"]))
    assert np.float32(el) == z["eval/loss"]
    m, lv = tr.encode(x)
    np.testing.assert_array_equal(m.numpy(), z["eval/enc_mean"])
    np.testing.assert_array_equal(lv.numpy(), z["eval/enc_lnvar"])


@pytest.mark.parametrize("path", golden_files("nb_"), ids=os.path.basename)
def test_kernel_algebra_matches_golden(path):
    """The analytic gradients the HIP kernels implement (f64) vs the golden fp32 autograd."""
    z = load(path)
    d = dims(z)
    P = {k: v.astype(np.float64) for k, v in params_of(z, "init/").items()}
    FR = {k: v.astype(np.float64) for k, v in params_of(z, "frozen/").items()}
    cells = z["s0/cells"]
    x = synth.densify(z["rowptr"], z["col"], z["val"], cells, d["D"]).astype(np.float64)
    L, G = nb_analytic.nb_step_grads(P, FR, x, z["covar"][cells].astype(np.float64),
                                     z["s0/eps_mu"].astype(np.float64), z["s0/eps_nu"].astype(np.float64),
                                     float(z["s0/beta"]), relu=relu_of(z))
    assert abs(L - float(z["s0/loss"])) / abs(L) < 1e-5
    for k in nb_oracle.param_names():
        want = z[f"s0/grad/{k}"].astype(np.float64).ravel()
        got = np.asarray(G[k], np.float64).ravel()
        assert np.abs(got - want).max() <= 2e-4 * np.abs(got).max() + 1e-7, k


def test_golden_fixtures_present():
    assert len(golden_files("nb_")) >= 5, GOLDEN


def test_kl_beta_schedule():
    # nb_loss_t (src/nb_vae_main.cc:26-32) with the mmvae defaults kl_max=1, kl_min=.01, discount=.1
    assert nb_oracle.kl_beta(0) == 1.0
    assert abs(nb_oracle.kl_beta(10) - np.exp(-1.0)) < 1e-6
    assert nb_oracle.kl_beta(1000) == np.float32(0.01)


def test_relu_hidden_encoder_rejected():
    # Q2: the reference throws at construction (nb.hh:334-337)
    with pytest.raises(ValueError):
        nb_oracle.init_params(10, enc_layers=(4,), relu=True)
