"""vMF-VAE oracle: the reference's op sequence on ATen CPU fp32 (test infrastructure only).

Restates ``include/models/vmf.hh:250-440``, the Angular layer
(``include/modules/angular.hh:34-70``) and the custom ``lbessel`` autograd op
(``include/operators.hh:13-101``).  As in the reference the *latent* is Gaussian; the
von Mises-Fisher distribution is the likelihood of the L2-normalised log1p data.
Quirks: Q3 (lbessel backward ignores the upstream gradient), Q4 (ln_kappa starts just below
kappa_min so the strict clamp mask zeroes its gradient), Q5 (fasterlog/fasterlgamma).
"""
from collections import OrderedDict
import math

import numpy as np
import torch
import torch.nn.functional as F

from .adam import LibTorchAdam, clip_grad_norm_
from .fastmath import fasterlgamma, fasterlog
from .nb_oracle import _linear_init

F32 = torch.float32


class _LBessel(torch.autograd.Function):
    """operators.hh:49-101 forward, operators.hh:20-40 backward."""

    @staticmethod
    def forward(ctx, kappa, nu):
        ctx.save_for_backward(kappa)
        ctx.nu = float(nu)
        nu = float(nu)
        eta = float(np.float32((nu + 0.5) / (2.0 * (nu + 1.0))))           # const float eta
        stuff1 = nu * torch.log(kappa) + eta * kappa - (eta + nu) * math.log(2.0) \
            - float(fasterlgamma(np.float32(nu + 1)))
        stuff2 = kappa - 0.5 * torch.log(kappa) - 0.5 * math.log(2.0 * math.pi)
        return torch.le(kappa, nu).type_as(kappa).mul(stuff1) + torch.gt(kappa, nu).type_as(kappa).mul(stuff2)

    @staticmethod
    def backward(ctx, grad):
        (x,) = ctx.saved_tensors
        df = ctx.nu
        lb = torch.sqrt(x * x * df / (df + 1.0) + df * df)
        ub = torch.sqrt(x * x + df * df)
        return 0.5 * (lb + ub) / x, None   # Q3: grad (the upstream) is not used


class _LBesselNoGrad(_LBessel):
    """The same forward with no backward contribution: the data-parallel restatement adds the
    upstream-independent Baricz gradient (Q3) on rank 0 only, so the ranks' summed gradient
    equals the single-process one."""

    @staticmethod
    def backward(ctx, grad):
        return torch.zeros_like(ctx.saved_tensors[0]), None


def lbessel_op(kappa, nu, with_grad=True):
    return (_LBessel if with_grad else _LBesselNoGrad).apply(kappa, nu)


def param_names():
    """vmf_vae_tImpl registration order (vmf.hh:325-388)."""
    return ["x_mean", "ln_x_sd", "ln_kappa", "covar_encoding.weight", "covar_encoding.bias",
            "representation_mean.weight", "representation_mean.bias",
            "representation_logvariance.weight", "representation_logvariance.bias",
            "covar_decoding_.weight", "covar_decoding_.bias"]


def init_params(D, C=1, Z=2, kappa_min=0.1, seed=0, enc_layers=(), dec_layers=()):
    """vmf_vae_tImpl::vmf_vae_tImpl (vmf.hh:307-389).  Hidden encoder layers are Angular layers
    named encoding_l (vmf.hh:338-345); without them one unnamed Angular maps to the latent
    ("z_enc.0", :348-355).  Hidden decoder layers are Linears decoding_l, then "decoding"."""
    g = torch.Generator().manual_seed(seed)
    p = OrderedDict()
    p["x_mean"] = torch.zeros((1, D), dtype=F32)
    p["ln_x_sd"] = torch.ones((1, D), dtype=F32)
    p["ln_kappa"] = torch.ones((1,), dtype=F32) * float(np.log(np.float32(kappa_min)))  # vmf.hh:323
    fr = OrderedDict()
    d_prev = D
    for l, dn in enumerate(enc_layers):  # Angular: kaiming_uniform_(a = sqrt 5), angular.hh:62
        fr[f"z_enc.encoding_{l + 1}.weight"] = (torch.rand((dn, d_prev), generator=g, dtype=F32) * 2 - 1) / math.sqrt(d_prev)
        d_prev = dn
    if len(enc_layers) < 1:
        fr["z_enc.0.weight"] = (torch.rand((Z, D), generator=g, dtype=F32) * 2 - 1) / math.sqrt(D)
        d_prev = Z
    p["covar_encoding.weight"], p["covar_encoding.bias"] = _linear_init(g, Z, C)
    p["representation_mean.weight"], p["representation_mean.bias"] = _linear_init(g, Z, d_prev)
    p["representation_logvariance.weight"], p["representation_logvariance.bias"] = _linear_init(g, Z, d_prev)
    d_prev = Z
    for l, dn in enumerate(dec_layers):
        fr[f"z_dec.decoding_{l + 1}.weight"], fr[f"z_dec.decoding_{l + 1}.bias"] = _linear_init(g, dn, d_prev)
        d_prev = dn
    fr["z_dec.decoding.weight"], fr["z_dec.decoding.bias"] = _linear_init(g, D, d_prev)
    p["covar_decoding_.weight"], p["covar_decoding_.bias"] = _linear_init(g, D, C)
    assert list(p.keys()) == param_names()
    return p, fr


def _vlayer_order(k):
    # "z_enc.encoding_1" < "encoding_2" < ...; the unnamed "z_enc.0" / final "z_dec.decoding" last
    tail = k.rsplit(".", 1)[1]
    if "_" in tail and tail.rsplit("_", 1)[1].isdigit():
        return (0, int(tail.rsplit("_", 1)[1]))
    return (1, 0)


class VMFModel:
    def __init__(self, params, frozen, kappa_min=0.1, kappa_max=10.0, relu=False):
        self.p = OrderedDict((k, v.clone().requires_grad_(True)) for k, v in params.items())
        self.fr = OrderedDict((k, v.clone()) for k, v in frozen.items())
        self.kmin, self.kmax = float(np.float32(kappa_min)), float(np.float32(kappa_max))
        self.relu = relu
        self.enc_keys = sorted({k.rsplit(".", 1)[0] for k in self.fr if k.startswith("z_enc.")}, key=_vlayer_order)
        self.dec_keys = sorted({k.rsplit(".", 1)[0] for k in self.fr if k.startswith("z_dec.")}, key=_vlayer_order)

    def lin(self, name, x):
        return F.linear(x, self.p[name + ".weight"], self.p[name + ".bias"])

    def angular(self, x, key="z_enc.0"):
        """angular.hh:34-42: W~ = normalize(relu(W) + 1e-4, dim=1); x W~^T (no bias)."""
        ww = F.normalize(F.relu(self.fr[key + ".weight"]) + 1e-4, p=2.0, dim=1)
        return F.linear(x, ww)

    def z_enc(self, x):
        """The Angular Sequential, a ReLU after every layer with --relu (vmf.hh:338-355)."""
        for k in self.enc_keys:
            x = self.angular(x, k)
            if self.relu:
                x = F.relu(x)
        return x

    def z_dec(self, z):
        """Hidden Linears (+ ReLU with --relu, vmf.hh:374-381), then the final "decoding"."""
        for i, k in enumerate(self.dec_keys):
            z = F.linear(z, self.fr[k + ".weight"], self.fr[k + ".bias"])
            if self.relu and i < len(self.dec_keys) - 1:
                z = F.relu(z)
        return z

    def encode(self, x, c=None):
        """vmf.hh:250-265 (with covariate) / vmf.hh:267-281 (recorder)."""
        eps = 1e-2 / float(np.float32(x.size(1)))
        xn = F.normalize(x.log1p(), p=2.0, dim=1)
        xn_std = torch.div(torch.sub(xn, self.p["x_mean"]), F.softplus(self.p["ln_x_sd"]) + eps)
        h = self.z_enc(xn_std)
        lnvar = torch.clamp(self.lin("representation_logvariance", h), -4.0, 4.0)
        mean = self.lin("representation_mean", h)
        if c is not None:
            mean = mean + self.lin("covar_encoding", c)
        return mean, lnvar

    def decode(self, z, c):
        """vmf.hh:283-290."""
        h = torch.exp(self.z_dec(z))
        hc = self.lin("covar_decoding_", c)
        return F.normalize(h + hc, p=2.0, dim=1)

    def forward(self, x, c, eps, training=True):
        """vmf.hh:292-304 (Gaussian reparameterisation vmf.hh:394-404)."""
        mean, lnvar = self.encode(x, c)
        z = mean + eps.mul(lnvar.div(2.0).exp()) if training else mean
        recon = self.decode(z, c)
        kappa = torch.clamp(torch.exp(self.p["ln_kappa"]), self.kmin, self.kmax)
        return dict(recon=recon, mean=mean, lnvar=lnvar, kappa=kappa)


def vmf_vae_loss(x, y, kl_weight, n_total=None, lbessel_grad=True):
    """vmf.hh:419-440.

    n_total / lbessel_grad (data-parallel restatement only): the divisor is the GLOBAL batch
    and only one rank carries the lbessel backward."""
    eps = 1e-2 / float(np.float32(x.size(1)))
    yobs = F.normalize(F.relu(x).log1p() + eps, p=2.0, dim=1)
    n = float(yobs.size(0)) if n_total is None else float(n_total)
    dd = float(yobs.size(1))
    df = float(np.float32(max(0.5 * dd - 1.0, 0.0)))
    kl = -0.5 * torch.sum(1 + y["lnvar"] - y["mean"].pow(2) - y["lnvar"].exp())
    llik = torch.sum(yobs * y["recon"], 1) * y["kappa"]
    llik = llik + (df * torch.log(y["kappa"]) - lbessel_op(y["kappa"], df, lbessel_grad))
    llik = llik - 0.5 * dd * float(fasterlog(np.float32(2.0 * math.pi)))
    return kl / n * kl_weight - llik.sum() / n


class VMFTrainer:
    def __init__(self, params, frozen, lr=1e-3, kappa_min=0.1, kappa_max=10.0, grad_clip=1.0, relu=False):
        self.m = VMFModel(params, frozen, kappa_min, kappa_max, relu=relu)
        self.adam = LibTorchAdam(list(self.m.p.values()), lr=lr, weight_decay=1e-4)
        self.grad_clip = grad_clip

    def step(self, x, c, eps, beta):
        y = self.m.forward(x, c, eps, True)
        L = vmf_vae_loss(x, y, beta)
        self.adam.zero_grad()
        L.backward()
        grads = OrderedDict((k, v.grad.detach().clone()) for k, v in self.m.p.items())
        total = clip_grad_norm_([v.grad for v in self.m.p.values()], self.grad_clip)
        self.adam.step()
        return dict(loss=float(L.detach()), grads=grads, total_norm=total)

    def step_dp(self, x, c, eps, beta, n_total, allreduce, rank):
        """The engine's data-parallel step (capi.hip mmvae_run, vmf_kernels.hip k_vgrad_small):
        this rank's rows, loss over the global batch, the lbessel backward on rank 0 only, SUM
        all-reduce of the registered gradients, then clip + Adam on every rank."""
        y = self.m.forward(x, c, eps, True)
        L = vmf_vae_loss(x, y, beta, n_total=n_total, lbessel_grad=(rank == 0))
        self.adam.zero_grad()
        L.backward()
        gl = [v.grad for v in self.m.p.values()]
        allreduce(gl)
        grads = OrderedDict((k, v.grad.detach().clone()) for k, v in self.m.p.items())
        total = clip_grad_norm_(gl, self.grad_clip)
        self.adam.step()
        return dict(loss=float(L.detach()), grads=grads, total_norm=total)

    @torch.no_grad()
    def eval_loss(self, x, c, eps, beta):
        return float(vmf_vae_loss(x, self.m.forward(x, c, eps, True), beta))

    @torch.no_grad()
    def encode(self, x):
        return self.m.encode(x, None)

    def params(self):
        return OrderedDict((k, v.detach().clone()) for k, v in self.m.p.items())
