"""CPU test of the drop-in C++ headers (include/mmvae/*.hh): a reference-style translation unit
— the option parsing of src/nb_vae_main.cc:43-49 and the lbessel op of include/operators.hh:49 —
compiled with g++ against the shim and the container's LibTorch, and run.  The shim's option
parsers and lbessel are header-only: the TU links LibTorch alone (a LibTorch program that also
linked the engine's libmmvae.so would load two HIP runtimes — torch's bundled one and
/opt/rocm's — which this test avoids; the engine is driven through its C-ABI from a separate
process or through mmvae_host).

Checks: the four option groups parse one argv exactly as the reference's parsers (defaults,
long-option aliases, the comma lists of --mean_encoding, Q7's ignored --grad_clip); the
lbessel forward equals the engine's host restatement; its backward returns the Baricz bound
whatever the upstream gradient is.
"""
import os
import subprocess

import numpy as np
import pytest

import mmvae_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

TU = r'''
#include "mmvae/options.hh"
#include "mmvae/operators.hh"
#include <cstdio>

int main(int argc, const char* argv[]) {
    using namespace mmvae::nb;          // as src/vmf_vae_main.cc:41 does for its model
    mmvae_options_t main_options;
    training_options_t train_opt;
    nbvae_options_t nb_opt;
    mmvae::vmf::vmf_options_t vmf_opt;
    if (parse_mmvae_options(argc, argv, main_options) != EXIT_SUCCESS) return 3;
    parse_nbvae_options(argc, argv, nb_opt);
    parse_vmf_options(argc, argv, vmf_opt);
    parse_training_options(argc, argv, train_opt);
    std::printf("mm %s %s %s %lld %g %g %g\n", main_options.out.c_str(), main_options.idx.c_str(),
                main_options.covar_idx.c_str(), (long long)main_options.batch_size, main_options.kl_discount,
                main_options.kl_min, main_options.kl_max);
    std::printf("tr %g %g %lld %lld %lld\n", train_opt.lr, train_opt.grad_clip, (long long)train_opt.nboot,
                (long long)train_opt.max_epoch, (long long)train_opt.recording);
    std::printf("nb %lld %lld %lld %d %zu", (long long)nb_opt.mean_latent, (long long)nb_opt.overdispersion_encoding,
                (long long)nb_opt.overdispersion_latent, (int)nb_opt.do_relu, nb_opt.mean_encoding_layers.size());
    for (auto v : nb_opt.mean_encoding_layers) std::printf(" %lld", (long long)v);
    std::printf("\nvmf %lld %g %g %d\n", (long long)vmf_opt.latent, vmf_opt.kappa_min, vmf_opt.kappa_max,
                (int)vmf_opt.do_relu);
    // operators.hh:49: lbessel with autograd; the backward ignores the upstream gradient (Q3)
    auto kappa = torch::tensor({0.5f, 5.f, 24.f, 30.f}).requires_grad_(true);
    auto lb = lbessel(kappa, 24.0);
    (lb * -3.0).sum().backward();
    for (int i = 0; i < 4; ++i)
        std::printf("lb %.9g %.9g %.9g\n", kappa[i].item<float>(), lb[i].item<float>(), kappa.grad()[i].item<float>());
    return 0;
}
'''


@pytest.mark.timeout(600)
def test_reference_style_tu_against_the_shim(tmp_path):
    import torch
    T = os.path.dirname(torch.__file__)
    src = tmp_path / "tu.cc"
    src.write_text(TU)
    exe = tmp_path / "tu"
    cmd = ["g++", "-std=c++17", "-O1", str(src), "-o", str(exe), "-I" + os.path.join(ROOT, "include"),
           "-I" + os.path.join(T, "include"), "-I" + os.path.join(T, "include", "torch", "csrc", "api", "include"),
           "-L" + os.path.join(T, "lib"), "-ltorch", "-ltorch_cpu", "-lc10",
           "-Wl,-rpath," + os.path.join(T, "lib"), "-D_GLIBCXX_USE_CXX11_ABI=1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=580)
    assert r.returncode == 0, r.stderr[-3000:]
    mtx = tmp_path / "x.mtx"
    mtx.write_text("%%MatrixMarket matrix coordinate integer general\n2 2 1\n1 1 1\n")
    argv = [str(exe), "--mtx", str(mtx), "--out", "OUT", "--batch", "64", "--kl_max", "2", "--mean-latent", "8",
            "--overdispersion_encoding", "3", "--mean_encoding", "128,64", "--relu", "--learning_rate", "0.01",
            "--grad_clip", "5", "--boot", "2", "--epoch", "7", "--latent", "5", "--kappa-max", "20"]
    r = subprocess.run(argv, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    out = {}
    lbs = []
    for ln in r.stdout.splitlines():
        t = ln.split()
        if t[0] == "lb":
            lbs.append([float(v) for v in t[1:]])
        else:
            out[t[0]] = t[1:]
    assert out["mm"] == ["OUT", str(mtx) + ".index", ".index", "64", "0.1", "0.01", "2"]
    assert out["tr"] == ["0.01", "1", "2", "7", "10"]                     # --grad_clip ignored (Q7)
    assert out["nb"] == ["8", "3", "1", "1", "2", "128", "64"]
    assert out["vmf"] == ["5", "0.1", "20", "1"]
    for kap, lb, g in lbs:
        assert lb == pytest.approx(mmvae_amd.lbessel(kap, 24.0), rel=1e-7, abs=1e-6)
        assert g == pytest.approx(mmvae_amd.lbessel_grad(kap, 24.0), rel=1e-7)  # not -3 x Baricz
    # the branch switch at kappa = df (operators.hh:79-80)
    assert lbs[2][1] == pytest.approx(mmvae_amd.lbessel(24.0, 24.0), rel=1e-7)
    # missing mtx: parse_mmvae_options returns EXIT_FAILURE (mmvae.hh:197)
    r = subprocess.run([str(exe), "--mtx", str(tmp_path / "nope"), "--out", "O"], capture_output=True, text=True)
    assert r.returncode == 3 and "missing mtx file" in r.stderr


def test_dropin_engine_header_compiles_with_the_c_abi(tmp_path):
    """mmvae/mmvae.hh (options + engine C-ABI + host runtime, torch-free) in a TU linked to the
    engine libraries: cfg from the reference's option structs, no GPU call."""
    src = tmp_path / "e.cc"
    src.write_text(r'''
#include "mmvae/mmvae.hh"
#include <cstdio>
int main(int argc, const char* argv[]) {
    mmvae_options_t mo; training_options_t tr; mmvae::nb::nbvae_options_t nb;
    parse_nbvae_options(argc, argv, nb); parse_training_options(argc, argv, tr);
    const mmvae_cfg c = mmvae_cfg_from_nb(nb, tr, 500, 1, mo.batch_size);
    std::printf("%lld %lld %lld %d %g %d\n", (long long)c.K, (long long)c.H, (long long)c.max_batch, c.relu, c.lr,
                c.n_enc_hidden);
    return 0;
}
''')
    lib = os.path.join(ROOT, "mm-vae_amd", "lib")
    exe = tmp_path / "e"
    r = subprocess.run(["g++", "-std=c++14", str(src), "-o", str(exe), "-I" + os.path.join(ROOT, "include"),
                        "-L" + lib, "-lmmvae_host", "-lmmvae", "-Wl,-rpath," + lib], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    r = subprocess.run([str(exe), "--mean_latent", "16", "--overdisp-encoding", "2", "--relu", "--rate", "0.5"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["16", "2", "100", "1", "0.5", "0"]


DEEP_TU = r'''
#include "mmvae/mmvae.hh"
#include <cstdio>
int main(int argc, const char* argv[]) {
    training_options_t tr; mmvae::nb::nbvae_options_t nb; mmvae::vmf::vmf_options_t vo;
    parse_nbvae_options(argc, argv, nb); parse_vmf_options(argc, argv, vo); parse_training_options(argc, argv, tr);
    const mmvae_cfg c = mmvae_cfg_from_nb(nb, tr, 500, 1, 100);
    const mmvae_cfg v = mmvae_cfg_from_vmf(vo, tr, 500, 1, 100);
    std::printf("nb %d", c.n_enc_hidden);
    for (int i = 0; i < c.n_enc_hidden && i < MMVAE_MAX_HIDDEN; ++i) std::printf(" %d", c.enc_hidden[i]);
    std::printf("\nnbdec %d", c.n_dec_hidden);
    for (int i = 0; i < c.n_dec_hidden && i < MMVAE_MAX_HIDDEN; ++i) std::printf(" %d", c.dec_hidden[i]);
    std::printf("\nvmf %d", v.n_enc_hidden);
    for (int i = 0; i < v.n_enc_hidden && i < MMVAE_MAX_HIDDEN; ++i) std::printf(" %d", v.enc_hidden[i]);
    mmvae_h h = nullptr;
    // the shape checks of mmvae_create run before it looks for a device: a valid deep cfg gets
    // as far as the device lookup (MMVAE_E_HIP here), a cfg over MMVAE_MAX_HIDDEN is MMVAE_E_ARG
    const int rc = mmvae_create(&c, 0, &h);
    std::printf("\ncreate %d %s\n", rc, rc == MMVAE_E_ARG ? mmvae_last_error(nullptr) : "");
    if (h) mmvae_destroy(h);
    return 0;
}
'''


@pytest.mark.parametrize("n_layers", [6, 16, 17])
def test_dropin_cfg_keeps_every_hidden_layer(tmp_path, n_layers):
    """mmvae_cfg_from_nb / _from_vmf copy every hidden width of a reference option struct (nb.hh:331-379,
    vmf.hh:338-385: any depth), up to MMVAE_MAX_HIDDEN; a deeper list reaches mmvae_create with its true
    count and is rejected there (MMVAE_E_ARG), never silently truncated."""
    src = tmp_path / "deep.cc"
    src.write_text(DEEP_TU)
    lib = os.path.join(ROOT, "mm-vae_amd", "lib")
    exe = tmp_path / "deep"
    r = subprocess.run(["g++", "-std=c++14", str(src), "-o", str(exe), "-I" + os.path.join(ROOT, "include"),
                        "-L" + lib, "-lmmvae_host", "-lmmvae", "-Wl,-rpath," + lib], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    widths = [64 + 8 * i for i in range(n_layers)]
    enc = ",".join(str(v) for v in widths)
    dec = ",".join(str(v) for v in reversed(widths[:5]))
    env = dict(os.environ, HIP_VISIBLE_DEVICES="")  # CPU container: no device in any case
    r = subprocess.run([str(exe), "--mean_encoding", enc, "--mean_decoding", dec, "--encoding", enc],
                       capture_output=True, text=True, timeout=60, env=env)
    assert r.returncode == 0, r.stderr
    out = {ln.split()[0]: ln.split()[1:] for ln in r.stdout.splitlines() if ln.strip()}
    kept = widths[:16]
    assert out["nb"] == [str(n_layers)] + [str(v) for v in kept]
    assert out["vmf"] == [str(n_layers)] + [str(v) for v in kept]
    assert out["nbdec"] == ["5"] + [str(v) for v in reversed(widths[:5])]
    rc = int(out["create"][0])
    if n_layers <= 16:
        assert rc == -2, out  # MMVAE_E_HIP: every shape check passed
    else:
        assert rc == -1 and "MMVAE_MAX_HIDDEN" in " ".join(out["create"][1:]), out

