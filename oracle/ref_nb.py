"""Driver of the reference's own NB-VAE (TEST INFRASTRUCTURE ONLY; this container only).

``oracle/_ref/ref_nb_harness`` is built by ``make -C oracle`` from
``/root/reference/include/models/nb.hh:1-563`` against this image's LibTorch 2.10 (see
``oracle/ref_nb_harness.cc``).  This module feeds it a dataset and a batch schedule and reads
back what the reference computed: its seeded parameter init, the noise its ``forward`` drew
(``nb.hh:462-472``, recovered bit-exactly), the loss (``nb.hh:539-548``), the pre-clip
gradients, the ``clip_grad_norm_`` total and the post-Adam parameters of every step
(``mmvae_alg.hh:290-310``), one eval forward (Q12) and the recorder's ``encode_mu(x)``.

``tests/golden/make_golden.py`` writes the NB golden fixtures from it, so every NB parity
test — the oracle's on the CPU and the HIP engine's on the GPU — compares against outputs
of the reference itself.  The GPU box never runs this (no ``/root/reference`` there).
"""
import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
HARNESS = os.path.join(HERE, "_ref", "ref_nb_harness")


def available():
    return os.access(HARNESS, os.X_OK)


def _read_out(d):
    out = {}
    with open(os.path.join(d, "out", "manifest.txt")) as f:
        for line in f:
            parts = line.split()
            key, dt, shape = parts[0], parts[1], tuple(int(s) for s in parts[2:])
            a = np.fromfile(os.path.join(d, "out", key.replace("/", "@") + ".bin"),
                            dtype=np.float64 if dt == "f64" else np.float32)
            out[key] = a.reshape(shape)
    return out


def run(D, C, K, H, R, relu, init_seed, enc_layers, dec_layers, steps, evalb, params_in=None):
    """Run the reference on a schedule.

    steps: list of dicts (x [B, D] f32 batch rows, c [B, C] f32, ridx [B] int64, beta, seed);
    evalb: dict (x, c, beta, seed).  params_in: optional {name: array} overriding the
    reference's seeded init (registered names; frozen as ``mu_enc.*`` / ``mu_dec.*``).
    Returns {key: array} with keys init/*, frozen/*, s{t}/{eps_mu,eps_nu,loss,total_norm,
    grad/*,param/*}, eval/{eps_mu,eps_nu,loss,enc_mean,enc_lnvar}."""
    if not available():
        raise RuntimeError("oracle/_ref/ref_nb_harness not built (make -C oracle, needs /root/reference)")
    with tempfile.TemporaryDirectory() as d:
        lines = [f"{D} {C} {K} {H} {R} {int(bool(relu))} {int(init_seed)}",
                 " ".join(str(v) for v in [len(enc_layers), *enc_layers]),
                 " ".join(str(v) for v in [len(dec_layers), *dec_layers]),
                 str(len(steps))]
        for t, s in enumerate(steps):
            x = np.ascontiguousarray(s["x"], np.float32)
            B = x.shape[0]
            assert x.shape == (B, D) and s["c"].shape == (B, C) and s["ridx"].shape == (B,)
            x.tofile(os.path.join(d, f"x{t}.f32"))
            np.ascontiguousarray(s["c"], np.float32).tofile(os.path.join(d, f"c{t}.f32"))
            np.ascontiguousarray(s["ridx"], np.int64).tofile(os.path.join(d, f"ridx{t}.i64"))
            lines.append(f"{B} {np.float32(s['beta']):.9g} {int(s['seed'])}")
        x = np.ascontiguousarray(evalb["x"], np.float32)
        x.tofile(os.path.join(d, "xe.f32"))
        np.ascontiguousarray(evalb["c"], np.float32).tofile(os.path.join(d, "ce.f32"))
        lines.append(f"{x.shape[0]} {np.float32(evalb['beta']):.9g} {int(evalb['seed'])}")
        with open(os.path.join(d, "spec.txt"), "w") as f:
            f.write("\n".join(lines) + "\n")
        if params_in:
            os.makedirs(os.path.join(d, "in"))
            for k, v in params_in.items():
                np.ascontiguousarray(v, np.float32).tofile(os.path.join(d, "in", k + ".f32"))
        subprocess.run([HARNESS, d], check=True)
        return _read_out(d)
