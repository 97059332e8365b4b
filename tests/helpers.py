"""Shared helpers for the parity tests (fixture loading, engine setup, comparisons)."""
import glob
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden_files(prefix="nb_"):
    return sorted(glob.glob(os.path.join(GOLDEN, prefix + "*.npz")))


def load(path):
    z = np.load(path)  # allow_pickle defaults to False
    return {k: z[k] for k in z.files}


def dims(z):
    return {k: int(z[k]) for k in ("N", "D", "K", "C", "H", "R", "B")}


def params_of(z, prefix):
    return {k[len(prefix):]: z[k] for k in z if k.startswith(prefix)}


def eps_of(z, tag):
    return np.concatenate([z[f"{tag}/eps_mu"].ravel(), z[f"{tag}/eps_nu"].ravel()]).astype(np.float32)


def model_of(z):
    return str(z["model"]) if "model" in z else "nb"


def relu_of(z):
    return bool(int(z["relu"])) if "relu" in z else False


def hidden_of(z):
    """(enc_layers, dec_layers) of a fixture: the frozen hidden widths (--mean_encoding ...)."""
    return tuple(int(v) for v in z.get("enc_layers", ())), tuple(int(v) for v in z.get("dec_layers", ()))


def engine_from_fixture(z, dtype="f32"):
    from mmvae_amd import MODEL_NB, MODEL_VMF, Engine
    d = dims(z)
    model = MODEL_VMF if model_of(z) == "vmf" else MODEL_NB
    enc, dec = hidden_of(z)
    eng = Engine(D=d["D"], K=d["K"], C=d["C"], H=d["H"], R=d["R"], max_batch=max(d["B"], 64), dtype=dtype,
                 model=model, relu=relu_of(z), enc_hidden=enc, dec_hidden=dec)
    eng.upload_csr(z["rowptr"], z["col"], z["val"], covar=z["covar"])
    eng.set_params(params_of(z, "init/"))
    eng.set_params(params_of(z, "frozen/"))
    return eng


def rel_err(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-30))


def assert_grads_close(got, want, rtol, ctx=""):
    """Norm-relative: max|got - want| <= rtol * max|want| per tensor."""
    bad = []
    for k, w in want.items():
        e = rel_err(got[k], w)
        if e > rtol:
            bad.append((k, e))
    assert not bad, f"{ctx} gradient mismatch (rtol {rtol}): {bad}"


def assert_adam_close(got, want, grads, lr=1e-3, atol=2e-5, ctx="", noisy_keys=()):
    """Post-Adam params.  Adam's first steps move every coordinate by ~lr*sign(g): a
    coordinate whose gradient is at the fp32 noise floor may flip sign, so those are
    allowed an lr-sized difference; all others must agree to atol."""
    bad = []
    for k, w in want.items():
        g = np.abs(np.asarray(grads[k], np.float64).ravel())
        d = np.abs(np.asarray(got[k], np.float64).ravel() - np.asarray(w, np.float64).ravel())
        noisy = g <= 1e-4 * (g.max() + 1e-30)
        if k in noisy_keys:
            noisy = np.ones_like(noisy)
        lim = np.where(noisy, 2.5 * lr, atol)
        if np.any(d > lim):
            i = int(np.argmax(d - lim))
            bad.append((k, float(d[i]), float(g[i])))
    assert not bad, f"{ctx} parameter mismatch after Adam: {bad}"


def kappa_grad_atol(D, kappa, record=None):
    """Absolute tolerance of the vMF ln_kappa gradient, from its f32 cancellation.

    d loss / d kappa holds two terms of size df / kappa that nearly cancel: the likelihood's
    -df (B / n) / kappa and the lbessel backward's Baricz bound (lb + ub) / (2 kappa) with
    lb, ub ~ df (operators.hh:33-35, vmf.hh:419-440); the difference is O(kappa / df).  The
    reference evaluates them in f32, and so do the oracle and the engine, each in its own order:
    every evaluation carries up to ~4 ulp of df / kappa (sqrt, product, sum, quotient), and the
    two being compared round independently, hence 8 ulp_f32(df / kappa), times kappa for the
    ln_kappa chain rule (d / d ln kappa = kappa d / d kappa).  At configs[2] (D = 20k, df = 9999,
    kappa = 4): 8 * 2^-12 * 4 = 7.8e-3."""
    df = max(0.5 * D - 1.0, 0.0)
    if df <= 0:
        return 1e-6
    t = df / kappa
    ulp = 2.0 ** (np.floor(np.log2(t)) - 23)
    atol = 8.0 * ulp * kappa
    if record is not None:
        record.append({"D": D, "kappa": kappa, "atol": atol})
    return atol


def record_kappa_err(tag, D, kappa, got, want, atol):
    """Appends the measured ln_kappa gradient difference to gpurun_out/kappa_grad_err.jsonl."""
    import json
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    d = os.path.join(root, "gpurun_out")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "kappa_grad_err.jsonl"), "a") as f:
        f.write(json.dumps({"test": tag, "D": int(D), "kappa": float(kappa), "got": float(got), "want": float(want),
                            "abs_err": abs(float(got) - float(want)), "atol": float(atol),
                            "rel_err": abs(float(got) - float(want)) / max(abs(float(want)), 1e-30)}) + "\n")
