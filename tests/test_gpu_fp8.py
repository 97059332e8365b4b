"""The fp8 e4m3 mode (BASELINE configs[4] "fp8 MFMA encoder/decoder", -m gpu): the decoder
logit GEMM z W_dec^T of all three decoder passes and the encoder GEMM log1p(x) (W_enc / sd)^T on
v_mfma_f32_16x16x32_fp8_fp8 (W_dec pre-scaled by a power of two to the top of the e4m3 range; the
encoder image W_enc / sd re-scaled every step by the power of two k_enc_scale bounds; z and
log1p(x) rounded to e4m3 as loaded / scattered; f32 accumulate); the backward (dz, encoder
dh^T log1p(x)) GEMMs stay bf16.  SURVEY §8(d) allows 1e-2 relative ELBO for fp8.  Checked against the oracle's golden
steps (every NB fixture) beside the bf16 mode's error, and at the configs[4] per-GPU shape
(D = 30000, B = 8192, latent 64) against the fp32-accurate bf16x3 mode.  The error table is
written to gpurun_out/fp8_accuracy.json.
"""
import json
import os

import numpy as np
import pytest

from helpers import assert_grads_close, engine_from_fixture, eps_of, golden_files, load, params_of, rel_err

pytestmark = pytest.mark.gpu

NB_FILES = golden_files("nb_")
TABLE = {}


def _grad_err(got, want):
    return max(rel_err(got[k], want[k]) for k in want)


@pytest.mark.parametrize("path", NB_FILES, ids=os.path.basename)
def test_fp8_against_oracle_fixtures(path):
    z = load(path)
    row = {}
    for dtype in ("bf16", "fp8"):
        eng = engine_from_fixture(z, dtype)
        loss, _ = eng.step(z["s0/cells"], float(z["s0/beta"]), eps=eps_of(z, "s0"))
        want = float(z["s0/loss"])
        row[dtype] = {"loss_rel": abs(loss - want) / abs(want), "grad_rel": _grad_err(eng.grads(), params_of(z, "s0/grad/"))}
    TABLE[os.path.basename(path)] = row
    assert row["fp8"]["loss_rel"] <= 1e-2, row  # fp8 ELBO within 1e-2 rel
    # gradients (documented, not parity): within 10 % norm-relative of the oracle on every
    # fixture with K > 1 (measured 3-5 %, profiles/r3_fp8_accuracy.json).  K = 1 fixtures (nb_k1,
    # nb_b64_k1_chr2) carry no gradient information at e4m3: the single encoder output is a sum of
    # a few 3-mantissa-bit products and each head weight is a 1 x 1 scalar, so their gradients are
    # recorded in the table (measured 35-99 %) and only required finite; their loss is held above
    assert np.isfinite(row["fp8"]["grad_rel"]), row
    if int(z["K"]) > 1:
        assert row["fp8"]["grad_rel"] <= 0.1, row


def test_fp8_configs4_shape_against_x3():
    """configs[4] per-GPU shape (1M x 30k model, B = 8192 / GPU): fp8 vs the parity-grade mode."""
    from mmvae_amd import Engine
    D, K, B = 30000, 64, 8192
    out = {}
    for dtype in ("bf16x3", "bf16", "fp8"):
        eng = Engine(D=D, K=K, max_batch=B, dtype=dtype, seed=3)
        eng.synth_csr(20000, lib_size=2000.0, seed=5)
        eng.init_params(seed=7)
        cells = np.random.default_rng(1).integers(0, 20000, B)
        loss, norm = eng.step(cells, 1.0, step_id=4)
        out[dtype] = (loss, norm, eng.grads())
    ref = out["bf16x3"]
    row = {}
    for dtype in ("bf16", "fp8"):
        loss, norm, g = out[dtype]
        row[dtype] = {"loss_rel": abs(loss - ref[0]) / abs(ref[0]), "norm_rel": abs(norm - ref[1]) / ref[1],
                      "grad_rel": _grad_err(g, ref[2])}
    TABLE["configs4_D30000_B8192_vs_bf16x3"] = row
    root = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
    with open(os.path.join(root, "gpurun_out", "fp8_accuracy.json"), "w") as f:
        json.dump(TABLE, f, indent=1)
    assert row["fp8"]["loss_rel"] <= 1e-2, row
    # at the shape the mode is for, gradients within 5 % (norm-relative) of the parity-grade mode
    assert row["fp8"]["grad_rel"] <= 5e-2, row
