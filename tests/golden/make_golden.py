"""Generate the golden NB/vMF fixtures (run in the build container only).

NB fixtures come from the reference itself (oracle/ref_nb.py, `make -C oracle` first);
vMF fixtures from the oracle restatement (the reference's vmf.hh cannot build on
LibTorch 2.10: operators.hh:45 calls the removed SavedVariable::reset_grad_function).

    python tests/golden/make_golden.py

Each fixture is a small .npz: the dataset CSR, per-step cell ids / covariates / noise /
beta, the initial registered and frozen parameters (LibTorch names), and per step the
oracle's loss, pre-clip gradients, clip total-norm and post-Adam parameters, plus one
eval-forward loss (Q12).  The oracle runs the reference's own call sequence on ATen 2.10
CPU fp32 (see oracle/__init__.py for why this pins parity).
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import nb_oracle, ref_nb, synth, vmf_oracle  # noqa: E402

NB_CASES = [
    # name, N, D, K, C, H, R, B, steps, lib, seed[, relu, enc_layers, dec_layers]
    ("nb_small", 40, 50, 8, 1, 1, 1, 16, 3, 200.0, 1),
    ("nb_mid", 300, 500, 16, 1, 1, 1, 64, 3, 300.0, 2),
    ("nb_generic", 60, 70, 5, 2, 2, 2, 32, 3, 150.0, 3),
    ("nb_k1", 20, 30, 1, 1, 1, 1, 8, 2, 100.0, 4),
    ("nb_dups", 10, 40, 8, 1, 1, 1, 24, 2, 120.0, 5),
    ("nb_k64", 128, 256, 64, 1, 1, 1, 128, 2, 500.0, 6),
    ("nb_relu", 100, 300, 16, 1, 1, 1, 64, 3, 300.0, 7, True),
    ("nb_hidden1", 100, 300, 16, 1, 1, 1, 64, 3, 300.0, 8, False, (24,), (20,)),
    ("nb_hidden2", 90, 200, 8, 2, 1, 1, 48, 3, 250.0, 9, False, (48, 12), (10, 40)),
    ("nb_hidden_relu", 90, 200, 16, 1, 1, 1, 48, 3, 250.0, 10, True, (), (32, 20)),
    # beyond the fused kernels' shape limits: the wide path (mm-vae_amd/csrc/wide.hip)
    ("nb_wide_k128", 100, 300, 128, 1, 1, 1, 64, 3, 300.0, 21),
    ("nb_wide_enc", 100, 300, 16, 1, 1, 1, 64, 3, 300.0, 22, False, (256, 128), (96,)),
    ("nb_wide_chr", 60, 120, 8, 12, 10, 9, 32, 3, 150.0, 23),
    ("nb_wide_deep", 80, 200, 8, 2, 1, 1, 48, 3, 250.0, 24, False, (40, 32, 24, 20, 16, 12), (10, 12, 14, 16, 18)),
    ("nb_wide_relu", 80, 200, 72, 1, 1, 1, 48, 3, 250.0, 25, True, (), (100, 80)),
    # the reference-pinning grid (B in {64, 256}, K in {1, 8, 64}, C = H = R in {1, 2}, duplicates)
    ("nb_b64_k1_chr2", 100, 200, 1, 2, 2, 2, 64, 3, 300.0, 41),
    ("nb_b64_k64_dups", 40, 300, 64, 1, 1, 1, 64, 3, 300.0, 42),
    ("nb_b256_k8", 300, 400, 8, 1, 1, 1, 256, 3, 400.0, 43),
    ("nb_b256_k64_chr2", 400, 600, 64, 2, 2, 2, 256, 3, 500.0, 44),
]


def make_nb(name, N, D, K, C, H, R, B, steps, lib, seed, relu=False, enc_layers=(), dec_layers=()):
    """Every number in an NB fixture is computed by the reference itself: its seeded
    parameter init, the noise its forward drew, loss, pre-clip gradients, clip norm,
    post-Adam parameters, the eval loss and encode_mu (oracle/ref_nb.py drives
    /root/reference/include/models/nb.hh:1-563 built on LibTorch 2.10).  This script only
    chooses the dataset (oracle/synth.py) and the batch schedule (mmvae_alg.hh:264-266,292-301)."""
    rowptr, col, val = synth.synth_csr(N, D, lib_size=lib, seed=seed)
    rng = np.random.default_rng(seed + 1000)
    if C == 1:
        covar = np.ones((N, 1), dtype=np.float32)  # nb_vae_main.cc:68-73 auto ones covariate
    else:
        covar = rng.standard_normal((N, C)).astype(np.float32)
    nbatch = (N + B - 1) // B
    sched, cells_of = [], []
    for t in range(steps):
        b = t % nbatch
        batch = (b * B + np.arange(B)) % N            # mmvae_alg.hh:264-266
        ridx = rng.integers(0, B, size=B)             # mmvae_alg.hh:292-293
        cells_of.append(batch[ridx])                  # index_select (mmvae_alg.hh:300-301)
        sched.append(dict(x=synth.densify(rowptr, col, val, batch, D), c=covar[batch], ridx=ridx,
                          beta=nb_oracle.kl_beta(t), seed=seed * 1000 + t))
    ecells = (np.arange(B) % N).astype(np.int64)      # one eval forward (Q12) on the first batch
    evalb = dict(x=synth.densify(rowptr, col, val, ecells, D), c=covar[ecells], beta=0.5, seed=seed * 1000 + 999)
    ref = ref_nb.run(D, C, K, H, R, relu, seed, enc_layers, dec_layers, sched, evalb)
    out = dict(N=N, D=D, K=K, C=C, H=H, R=R, B=B, steps=steps, relu=np.int32(relu),
               enc_layers=np.array(enc_layers, np.int32), dec_layers=np.array(dec_layers, np.int32),
               rowptr=rowptr, col=col, val=val, covar=covar,
               source=np.array("reference nb.hh:1-563 on LibTorch 2.10 (oracle/ref_nb_harness.cc)"))
    out.update(ref)
    for t in range(steps):
        out[f"s{t}/cells"] = cells_of[t].astype(np.int64)
        out[f"s{t}/beta"] = np.float32(sched[t]["beta"])
        out[f"s{t}/torch_seed"] = np.int64(sched[t]["seed"])
        out[f"s{t}/loss"] = np.float32(out[f"s{t}/loss"])
        out[f"s{t}/total_norm"] = np.float64(out[f"s{t}/total_norm"])
    out["eval/cells"] = ecells
    out["eval/beta"] = np.float32(0.5)
    out["eval/torch_seed"] = np.int64(evalb["seed"])
    out["eval/loss"] = np.float32(out["eval/loss"])
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **out)
    print(name, "loss", [float(out[f"s{t}/loss"]) for t in range(steps)], os.path.getsize(path), "bytes")


VMF_CASES = [
    # name, N, D, Z, C, B, steps, lib, seed, ln_kappa (None = reference init log(kappa_min), Q4)
    ("vmf_small", 40, 50, 8, 1, 16, 3, 200.0, 11, None),
    ("vmf_generic", 60, 70, 5, 2, 32, 3, 150.0, 12, float(np.log(np.float32(2.0)))),
    ("vmf_k32", 128, 256, 32, 1, 128, 2, 500.0, 13, float(np.log(np.float32(5.0)))),
    ("vmf_dups", 10, 40, 8, 1, 24, 2, 120.0, 14, float(np.log(np.float32(0.7)))),
    ("vmf_z64", 100, 300, 64, 1, 64, 2, 400.0, 15, float(np.log(np.float32(9.0)))),
    ("vmf_relu", 100, 300, 16, 1, 64, 3, 300.0, 16, float(np.log(np.float32(3.0))), True),
    ("vmf_hidden1", 100, 300, 16, 1, 64, 3, 300.0, 17, float(np.log(np.float32(3.0))), False, (24,), (20,)),
    ("vmf_hidden_relu", 90, 200, 8, 2, 48, 3, 250.0, 18, float(np.log(np.float32(2.0))), True, (40, 12), (10, 30)),
    # the wide path
    ("vmf_wide_z96", 100, 300, 96, 1, 64, 3, 400.0, 31, float(np.log(np.float32(4.0)))),
    ("vmf_wide_enc", 100, 300, 16, 1, 64, 3, 300.0, 32, float(np.log(np.float32(3.0))), True, (256, 100), (80,)),
    ("vmf_wide_deep", 80, 200, 8, 12, 48, 3, 250.0, 33, float(np.log(np.float32(2.0))), False, (40, 32, 24, 20, 16), (10, 12, 14, 16, 18)),
]


def make_vmf(name, N, D, Z, C, B, steps, lib, seed, ln_kappa, relu=False, enc_layers=(), dec_layers=()):
    rowptr, col, val = synth.synth_csr(N, D, lib_size=lib, seed=seed)
    rng = np.random.default_rng(seed + 1000)
    if C == 1:
        covar = np.ones((N, 1), dtype=np.float32)  # vmf_vae_main.cc auto ones covariate
    else:
        covar = rng.standard_normal((N, C)).astype(np.float32)
    params, frozen = vmf_oracle.init_params(D, C=C, Z=Z, seed=seed, enc_layers=enc_layers, dec_layers=dec_layers)
    if ln_kappa is not None:
        params["ln_kappa"] = torch.tensor([ln_kappa], dtype=torch.float32)
    tr = vmf_oracle.VMFTrainer(params, frozen, relu=relu)
    out = dict(N=N, D=D, K=Z, C=C, H=1, R=1, B=B, steps=steps, model="vmf", relu=np.int32(relu),
               enc_layers=np.array(enc_layers, np.int32), dec_layers=np.array(dec_layers, np.int32),
               rowptr=rowptr, col=col, val=val, covar=covar)
    for k, v in params.items():
        out["init/" + k] = v.numpy()
    for k, v in frozen.items():
        out["frozen/" + k] = v.numpy()
    nbatch = (N + B - 1) // B
    for t in range(steps):
        b = t % nbatch
        batch = (b * B + np.arange(B)) % N            # mmvae_alg.hh:264-266
        ridx = rng.integers(0, B, size=B)             # mmvae_alg.hh:292-293
        cells = batch[ridx]
        x = torch.from_numpy(synth.densify(rowptr, col, val, cells, D))
        c = torch.from_numpy(covar[cells])
        eps = torch.from_numpy(rng.standard_normal((B, Z)).astype(np.float32))
        beta = nb_oracle.kl_beta(t)
        r = tr.step(x, c, eps, beta)
        out[f"s{t}/cells"] = cells.astype(np.int64)
        out[f"s{t}/eps_mu"] = eps.numpy()
        out[f"s{t}/eps_nu"] = np.zeros((B, 0), np.float32)
        out[f"s{t}/beta"] = np.float32(beta)
        out[f"s{t}/loss"] = np.float32(r["loss"])
        out[f"s{t}/total_norm"] = np.float64(r["total_norm"])
        for k, v in r["grads"].items():
            out[f"s{t}/grad/" + k] = v.numpy()
        for k, v in tr.params().items():
            out[f"s{t}/param/" + k] = v.numpy()
    cells = (np.arange(B) % N).astype(np.int64)
    x = torch.from_numpy(synth.densify(rowptr, col, val, cells, D))
    c = torch.from_numpy(covar[cells])
    eps = torch.from_numpy(rng.standard_normal((B, Z)).astype(np.float32))
    out["eval/cells"] = cells
    out["eval/eps_mu"] = eps.numpy()
    out["eval/eps_nu"] = np.zeros((B, 0), np.float32)
    out["eval/beta"] = np.float32(0.5)
    out["eval/loss"] = np.float32(tr.eval_loss(x, c, eps, 0.5))
    m, lv = tr.encode(x)
    out["eval/enc_mean"] = m.numpy()
    out["eval/enc_lnvar"] = lv.numpy()
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **out)
    print(name, "loss", [float(out[f"s{t}/loss"]) for t in range(steps)], os.path.getsize(path), "bytes")


if __name__ == "__main__":
    torch.set_num_threads(1)
    which = sys.argv[1:] or ["nb", "vmf"]
    for case in NB_CASES:
        if "nb" in which or case[0] in which:
            make_nb(*case)
    for case in VMF_CASES:
        if "vmf" in which or case[0] in which:
            make_vmf(*case)
