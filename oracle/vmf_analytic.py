"""float64 numpy restatement of the *kernel algebra* of the vMF ELBO step (test infrastructure).

The HIP path (``mm-vae_amd/csrc/vmf_kernels.hip``) does not run autograd: it evaluates
hand-derived gradients of the reference's vMF forward/loss (``include/models/vmf.hh:250-440``,
``include/modules/angular.hh:34-42``, ``include/operators.hh:13-101``) restructured for the
GPU.  This module restates that algebra on the CPU so the CPU suite proves it equals LibTorch
autograd of the oracle (``oracle/vmf_oracle.py``) before anything runs on a GPU.  Each block
names the kernel that implements it.

Row quantities (cell b, l = log1p(x) on the nonzeros, eps = 1e-2/D):
  nx = max(||l||, 1e-12)                      F::normalize of log1p(x)       (vmf.hh:253)
  ny = max(sqrt(sum_g (l_g + eps)^2), 1e-12)  F::normalize of log1p(relu x)+eps (vmf.hh:422-423)
  v  = exp(W_d z + b_d) + W_cd c + b_cd,  nv = max(||v||, 1e-12),  r = v / nv  (vmf.hh:283-289)
  cos = <y, r> = (sum_nnz l v + eps sum_g v) / (ny nv)
The decoder backward of L = -(kappa/n) sum_b cos_b + ... is
  dv_bg = alpha_b (l_bg + eps) + beta_b v_bg,  alpha = -(kappa/n) / (nv ny),  beta = (kappa/n) cos / nv^2
and the encoder split is h = (l/nx) (W~/s)^T - (x_mean/s) W~^T, s = softplus(ln_x_sd) + eps.
"""
import math

import numpy as np

from .fastmath import fasterlgamma, fasterlog


def softplus(v):
    return np.where(v > 20.0, v, np.log1p(np.exp(np.minimum(v, 20.0))))


def dsoftplus(v):
    return np.where(v > 20.0, 1.0, 1.0 / (1.0 + np.exp(-v)))


def lbessel_fwd(kappa, nu):
    """operators.hh:65-81 in float64 (fasterlgamma as the reference evaluates it)."""
    eta = (nu + 0.5) / (2.0 * (nu + 1.0))
    s1 = nu * math.log(kappa) + eta * kappa - (eta + nu) * math.log(2.0) - float(fasterlgamma(np.float32(nu + 1)))
    s2 = kappa - 0.5 * math.log(kappa) - 0.5 * math.log(2.0 * math.pi)
    return s1 if kappa <= nu else s2


def lbessel_bwd(kappa, nu):
    """operators.hh:34-37: the Baricz bound, independent of the upstream gradient (Q3)."""
    lb = math.sqrt(kappa * kappa * nu / (nu + 1.0) + nu * nu)
    ub = math.sqrt(kappa * kappa + nu * nu)
    return 0.5 * (lb + ub) / kappa


def vmf_step_grads(P, FR, x, c, eps, beta, kappa_min=0.1, kappa_max=10.0, n_total=None, relu=False):
    """Loss and pre-clip gradients of every registered vMF parameter (kernel algebra)."""
    B, D = x.shape
    n = float(B if n_total is None else n_total)
    epsD = 1e-2 / D
    df = max(0.5 * D - 1.0, 0.0)
    from .vmf_oracle import _vlayer_order
    # frozen Sequentials (vmf.hh:338-385): Angular encoder layers (the first, D -> w0, is the big
    # GEMM; the rest a chain in k_vlatent_fwd, ReLU after each with --relu), hidden decoder
    # Linears (+ ReLU) before the final big decoder GEMM
    enc = sorted({k.rsplit(".", 1)[0] for k in FR if k.startswith("z_enc.")}, key=_vlayer_order)
    dec = sorted({k.rsplit(".", 1)[0] for k in FR if k.startswith("z_dec.")}, key=_vlayer_order)
    W = FR[enc[0] + ".weight"]
    Wd, bd = FR[dec[-1] + ".weight"], FR[dec[-1] + ".bias"]

    # ---- k_vnorm_enc (frozen prep): W~ = normalize(relu(W) + 1e-4) --------------------------
    def angular_w(Wa):
        Wr_ = np.maximum(Wa, 0.0) + 1e-4
        return Wr_ / np.maximum(np.sqrt((Wr_ * Wr_).sum(1, keepdims=True)), 1e-12)
    Wt = angular_w(W)
    enc_chain = [angular_w(FR[k + ".weight"]) for k in enc[1:]]
    dec_chain = [(FR[k + ".weight"], FR[k + ".bias"]) for k in dec[:-1]]

    # ---- k_vprep / k_vmvec -----------------------------------------------------------------
    th = P["ln_x_sd"][0]
    s = softplus(th) + epsD
    inv = 1.0 / s
    xm = P["x_mean"][0]
    mvec = Wt @ (xm * inv)

    # ---- row norms (dataset index cellnorm) ---------------------------------------------------------------
    l = np.log1p(x)
    ly = np.log1p(np.maximum(x, 0.0))
    nx = np.maximum(np.sqrt((l * l).sum(1)), 1e-12)
    ny = np.maximum(np.sqrt(((ly + epsD) ** 2).sum(1)), 1e-12)

    # ---- k_enc_fwd + k_vlatent_fwd -------------------------------------------------------------
    h = ((l * inv) @ Wt.T) / nx[:, None] - mvec
    if relu:                                          # vmf.hh:351-352: ReLU after Angular
        h = np.maximum(h, 0.0)
    hs = [h]                                          # frozen Angular chain (ReLU with --relu)
    for Wc in enc_chain:
        hs.append(hs[-1] @ Wc.T)
        if relu:
            hs[-1] = np.maximum(hs[-1], 0.0)
    h = hs[-1]
    mean = h @ P["representation_mean.weight"].T + P["representation_mean.bias"] \
        + c @ P["covar_encoding.weight"].T + P["covar_encoding.bias"]
    a = h @ P["representation_logvariance.weight"].T + P["representation_logvariance.bias"]
    lnvar = np.clip(a, -4, 4)
    sg = np.exp(lnvar / 2)
    z = mean + eps * sg
    zs = [z]                                          # frozen decoder chain (ReLU with --relu)
    for Wc, bc in dec_chain:
        zs.append(zs[-1] @ Wc.T + bc)
        if relu:
            zs[-1] = np.maximum(zs[-1], 0.0)
    kl = -0.5 * np.sum(1 + lnvar - mean ** 2 - np.exp(lnvar))

    # ---- k_vkappa ----------------------------------------------------------------------------
    lk = float(P["ln_kappa"][0])
    e = math.exp(lk)
    kap = min(max(e, kappa_min), kappa_max)
    kmask = 1.0 if (kappa_min <= e <= kappa_max) else 0.0
    T = df * math.log(kap) - lbessel_fwd(kap, df)
    c2 = 0.5 * D * float(fasterlog(np.float32(2.0 * math.pi)))

    # ---- k_vdec<0> + k_vrowfin -----------------------------------------------------------------
    u = np.exp(zs[-1] @ Wd.T + bd)
    v = u + c @ P["covar_decoding_.weight"].T + P["covar_decoding_.bias"]
    nvr = np.sqrt((v * v).sum(1))
    nv = np.maximum(nvr, 1e-12)
    cos = ((ly * v).sum(1) + epsD * v.sum(1)) / (ny * nv)
    llik = kap * cos + T - c2
    loss = kl / n * beta - llik.sum() / n

    kn = kap / n
    alpha = np.where(nvr >= 1e-12, -kn / (nv * ny), -kn / (1e-12 * ny))
    bet = np.where(nvr >= 1e-12, kn * cos / (nv * nv), 0.0)

    # ---- k_vdec<1>: dv, da, column sums, dz ----------------------------------------------------
    dv = alpha[:, None] * (ly + epsD) + bet[:, None] * v
    da = dv * u
    G = {}
    G["covar_decoding_.bias"] = dv.sum(0)
    G["covar_decoding_.weight"] = dv.T @ c
    dz = da @ Wd
    for i in range(len(dec_chain) - 1, -1, -1):
        if relu:
            dz = dz * (zs[i + 1] > 0)
        dz = dz @ dec_chain[i][0]

    # ---- k_vlatent_bwd -------------------------------------------------------------------------
    bn = beta / n
    dmean = dz + bn * mean
    dlnvar = dz * eps * sg * 0.5 + bn * 0.5 * (np.exp(lnvar) - 1.0)
    dA = np.where((a >= -4) & (a <= 4), dlnvar, 0.0)
    G["representation_mean.weight"] = dmean.T @ h
    G["representation_mean.bias"] = dmean.sum(0)
    G["representation_logvariance.weight"] = dA.T @ h
    G["representation_logvariance.bias"] = dA.sum(0)
    G["covar_encoding.weight"] = dmean.T @ c
    G["covar_encoding.bias"] = dmean.sum(0)
    dh = dmean @ P["representation_mean.weight"] + dA @ P["representation_logvariance.weight"]
    for i in range(len(enc_chain) - 1, -1, -1):
        if relu:
            dh = dh * (hs[i + 1] > 0)
        dh = dh @ enc_chain[i]
    if relu:
        dh = dh * (hs[0] > 0)

    # ---- k_enc_bwd (dh / nx against log1p x) + k_vgrad_genes -----------------------------------
    Gl = ((dh / nx[:, None]).T @ l * Wt).sum(0)      # sum_k W~[k,g] sum_b dh_bk l_bg / nx_b
    gs = dh.sum(0) @ Wt                             # sum_k cdh_k W~[k,g]
    G["x_mean"] = (-inv * gs)[None, :]
    G["ln_x_sd"] = (-(inv * inv) * (Gl - xm * gs) * dsoftplus(th))[None, :]

    # ---- k_vgrad_small: ln_kappa ---------------------------------------------------------------
    dk = -cos.sum() / n - (B / n) * df / kap + lbessel_bwd(kap, df)
    G["ln_kappa"] = np.array([dk * e * kmask])
    return loss, G
