"""NB-VAE oracle: the reference's op sequence on ATen CPU fp32 (test infrastructure only).

Every function restates ``/root/reference/include/models/nb.hh`` op for op (file:line in
each docstring) so that LibTorch autograd produces the reference's gradients.  Parameters
are plain leaf tensors keyed by their LibTorch ``named_parameters()`` names.

Parity-critical quirks reproduced:
  Q1  ``mu_enc``/``mu_dec`` are never ``register_module``'d (nb.hh:264,273,331-379): they
      are *frozen* — excluded from clip and Adam.  They live in ``frozen`` here.
  Q2  ``--relu`` with >=1 hidden encoder layer throws at construction (nb.hh:334-337).
  Q12 the per-batch reported loss is an extra train-mode forward (mmvae_alg.hh:277-285).
"""
from collections import OrderedDict
import math
import torch
import torch.nn.functional as F

from .adam import LibTorchAdam, clip_grad_norm_

F32 = torch.float32


def _linear_init(gen, out_f, in_f, bias=True):
    """torch::nn::Linear::reset_parameters: kaiming_uniform_(a=sqrt(5)) == U(+-1/sqrt(fan_in))."""
    bound = 1.0 / math.sqrt(in_f) if in_f > 0 else 0.0
    w = (torch.rand((out_f, in_f), generator=gen, dtype=F32) * 2 - 1) * bound
    b = (torch.rand((out_f,), generator=gen, dtype=F32) * 2 - 1) * bound if bias else None
    return w, b


def param_names(enc_layers=(), K=2, C=1, H=1, R=1):
    """LibTorch registration order of ``nbvae_tImpl`` (nb.hh:318-400): own params, then modules."""
    names = ["x_mean", "ln_x_sd", "mu_bias", "nu_bias"]
    for mod in ["covar_encoding", "mu_representation_mean", "mu_representation_logvariance",
                "covar_decoding", "nu_encoding", "nu_representation_mean",
                "nu_representation_logvariance", "nu_decoding", "depth"]:
        names += [mod + ".weight", mod + ".bias"]
    return names


def init_params(D, C=1, K=2, H=1, R=1, enc_layers=(), dec_layers=(), relu=False, seed=0):
    """Construct parameters as ``nbvae_tImpl::nbvae_tImpl`` does (nb.hh:299-401).

    Returns (params: OrderedDict registered, frozen: OrderedDict unregistered Sequentials).
    Random draws use a seeded torch.Generator (the reference is unseeded, Q6).
    """
    if relu and len(enc_layers) > 0:
        # nb.hh:334-337 pushes the Linear and the ReLU under the same name -> LibTorch throws.
        raise ValueError("Submodule 'mu_encoding_1' already defined (reference nb.hh:334-337)")
    g = torch.Generator().manual_seed(seed)
    p = OrderedDict()
    p["x_mean"] = torch.zeros((1, D), dtype=F32)
    p["ln_x_sd"] = torch.ones((1, D), dtype=F32)
    p["mu_bias"] = torch.zeros((1, D), dtype=F32)
    p["nu_bias"] = torch.zeros((1, D), dtype=F32)
    fr = OrderedDict()
    d_prev = D
    for l, dn in enumerate(enc_layers):
        w, b = _linear_init(g, dn, d_prev)
        fr[f"mu_enc.mu_encoding_{l + 1}.weight"], fr[f"mu_enc.mu_encoding_{l + 1}.bias"] = w, b
        d_prev = dn
    if len(enc_layers) < 1:
        w, b = _linear_init(g, K, d_prev)
        fr["mu_enc.mu_encoding.weight"], fr["mu_enc.mu_encoding.bias"] = w, b
        d_prev = K
    p["covar_encoding.weight"], p["covar_encoding.bias"] = _linear_init(g, K, C)
    p["mu_representation_mean.weight"], p["mu_representation_mean.bias"] = _linear_init(g, K, d_prev)
    p["mu_representation_logvariance.weight"], p["mu_representation_logvariance.bias"] = _linear_init(g, K, d_prev)
    d_prev = K
    for l, dn in enumerate(dec_layers):
        w, b = _linear_init(g, dn, d_prev)
        fr[f"mu_dec.mu_decoding_{l + 1}.weight"], fr[f"mu_dec.mu_decoding_{l + 1}.bias"] = w, b
        d_prev = dn
    w, b = _linear_init(g, D, d_prev)
    fr["mu_dec.mu_decoding.weight"], fr["mu_dec.mu_decoding.bias"] = w, b
    p["covar_decoding.weight"], p["covar_decoding.bias"] = _linear_init(g, D, C)
    p["nu_encoding.weight"], p["nu_encoding.bias"] = _linear_init(g, H, D)
    p["nu_representation_mean.weight"], p["nu_representation_mean.bias"] = _linear_init(g, R, H)
    p["nu_representation_logvariance.weight"], p["nu_representation_logvariance.bias"] = _linear_init(g, R, H)
    p["nu_decoding.weight"], p["nu_decoding.bias"] = _linear_init(g, D, R)
    p["depth.weight"], p["depth.bias"] = _linear_init(g, 1, D)
    assert list(p.keys()) == param_names()
    return p, fr


class NBModel:
    """Functional restatement of ``nbvae_tImpl`` (nb.hh:212-508)."""

    def __init__(self, params, frozen, relu=False):
        self.p = OrderedDict((k, v.clone().requires_grad_(True)) for k, v in params.items())
        # frozen Sequentials: autograd still flows *through* them (Q1) but they never update.
        self.fr = OrderedDict((k, v.clone()) for k, v in frozen.items())
        self.relu = relu
        self.enc_keys = sorted({k.rsplit(".", 1)[0] for k in self.fr if k.startswith("mu_enc.")},
                               key=_layer_order)
        self.dec_keys = sorted({k.rsplit(".", 1)[0] for k in self.fr if k.startswith("mu_dec.")},
                               key=_layer_order)

    def _seq(self, keys, x, final_relu):
        for i, k in enumerate(keys):
            x = F.linear(x, self.fr[k + ".weight"], self.fr[k + ".bias"])
            last = i == len(keys) - 1
            if self.relu and (not last or final_relu):
                x = F.relu(x)
        return x

    def lin(self, name, x):
        return F.linear(x, self.p[name + ".weight"], self.p[name + ".bias"])

    def encode_mu(self, x, c=None):
        """nb.hh:403-417 (with covariate) / nb.hh:419-431 (recorder, no covariate)."""
        eps = 1e-4
        x_sd = F.softplus(self.p["ln_x_sd"])
        xn_std = torch.div(x.log1p() - self.p["x_mean"], x_sd + eps)
        # nb.hh:342-347: with no hidden layers the ReLU (if any) follows the final Linear.
        h = self._seq(self.enc_keys, xn_std, final_relu=(len(self.enc_keys) == 1))
        ln_var_clamp = torch.clamp(self.lin("mu_representation_logvariance", h), -4.0, 4.0)
        mean = self.lin("mu_representation_mean", h)
        if c is not None:
            mean = mean + self.lin("covar_encoding", c)
        return mean, ln_var_clamp

    def decode_mu(self, z, c):
        """nb.hh:433-442: p = exp(log_softmax(mu_dec(z) + covar_dec(c) + mu_bias, 1))."""
        h = self._seq(self.dec_keys, z, final_relu=False)
        hc = self.lin("covar_decoding", c)
        logit_mu = torch.log_softmax(h + hc + self.p["mu_bias"], 1)
        return torch.exp(logit_mu)

    def encode_nu(self, x):
        """nb.hh:444-451 (raw x, no log1p)."""
        h = self.lin("nu_encoding", x)
        ln_var_clamp = torch.clamp(self.lin("nu_representation_logvariance", h), -4.0, 4.0)
        return self.lin("nu_representation_mean", h), ln_var_clamp

    def decode_nu(self, z):
        """nb.hh:453-460: clamp(softplus(nu_dec(z) - nu_bias), 1e-4, 1e4)."""
        ret = F.softplus(self.lin("nu_decoding", z) - self.p["nu_bias"])
        return torch.clamp(ret, 1e-4, 1e4)

    @staticmethod
    def reparameterize(mu, lnvar, eps, training=True):
        """nb.hh:462-472: mu + eps * exp(lnvar / 2); eps injected (randn_like in the reference)."""
        if not training:
            return mu
        sig = lnvar.div(2.0).exp()
        return mu + eps.mul(sig)

    def forward(self, x, c, eps_mu, eps_nu, training=True):
        """nb.hh:474-508.  eps order per forward: mu [B,K] then nu [B,R] (nb.hh:480-492)."""
        mu_mean, mu_lnvar = self.encode_mu(x, c)
        mu_ = self.decode_mu(self.reparameterize(mu_mean, mu_lnvar, eps_mu, training), c)
        nu_mean, nu_lnvar = self.encode_nu(x)
        nu_ = self.decode_nu(self.reparameterize(nu_mean, nu_lnvar, eps_nu, training))
        d_ = F.softplus(self.lin("depth", x))
        return dict(recon_mu=mu_, recon_nu=nu_, recon_depth=d_, mu_mean=mu_mean,
                    mu_lnvar=mu_lnvar, nu_mean=nu_mean, nu_lnvar=nu_lnvar)

    def registered(self):
        return list(self.p.values())


def _layer_order(k):
    # "mu_enc.mu_encoding_1" < "mu_enc.mu_encoding_2" < ... ; bare "mu_encoding" (no hidden) first
    tail = k.rsplit(".", 1)[1]
    if "_" in tail and tail.rsplit("_", 1)[1].isdigit():
        return (0, int(tail.rsplit("_", 1)[1]))
    return (1, 0)


def nllik_loss(x, y):
    """nb.hh:510-531 — negative NB log-likelihood summed over [B,D]."""
    eps = 1e-4
    nu = y["recon_nu"] + eps
    mu = y["recon_mu"] * y["recon_depth"] + eps
    lg = torch.lgamma(nu) + torch.lgamma(x + 1.0)
    lg = lg - torch.lgamma(nu + x)
    denom = torch.log(mu + nu)
    pr = x.mul(denom - torch.log(mu))
    pr = pr + nu.mul(denom - torch.log(nu))
    return torch.sum(lg + pr)


def kl_loss(mean, lnvar):
    """nb.hh:533-537."""
    return -0.5 * torch.sum(1 + lnvar - mean.pow(2) - lnvar.exp())


def loss(x, y, kl_weight=1.0, n_total=None):
    """nb.hh:539-548: (NLL + w*KL_mu + w*KL_nu) / n.

    n_total (data-parallel restatement only): the divisor is the GLOBAL batch, so the
    per-rank losses and gradients sum to the single-process ones."""
    recon = nllik_loss(x, y)
    n = float(x.size(0)) if n_total is None else float(n_total)
    ret = recon
    ret = ret + kl_loss(y["mu_mean"], y["mu_lnvar"]) * kl_weight
    ret = ret + kl_loss(y["nu_mean"], y["nu_lnvar"]) * kl_weight
    return ret / n


def kl_beta(epoch, kl_max=1.0, kl_min=1e-2, kl_discount=0.1):
    """nb_loss_t (src/nb_vae_main.cc:26-32): max(kl_max * exp(-discount * epoch), kl_min), float32."""
    import numpy as np
    rate = np.float32(kl_max) * np.exp(-np.float32(kl_discount) * np.float32(epoch))
    return float(max(np.float32(rate), np.float32(kl_min)))


class NBTrainer:
    """One reference ELBO step (mmvae_alg.hh:300-310) on the oracle model."""

    def __init__(self, params, frozen, lr=1e-3, relu=False, grad_clip=1.0):
        self.m = NBModel(params, frozen, relu=relu)
        self.adam = LibTorchAdam(self.m.registered(), lr=lr, weight_decay=1e-4)
        self.grad_clip = grad_clip

    def step(self, x, c, eps_mu, eps_nu, beta):
        """forward -> loss -> zero_grad -> backward -> clip_grad_norm_ -> adam.step.

        Returns dict(loss, grads (pre-clip, OrderedDict), total_norm)."""
        y = self.m.forward(x, c, eps_mu, eps_nu, True)
        L = loss(x, y, beta)
        self.adam.zero_grad()
        L.backward()
        grads = OrderedDict((k, v.grad.detach().clone()) for k, v in self.m.p.items())
        total = clip_grad_norm_([v.grad for v in self.m.p.values()], self.grad_clip)
        self.adam.step()
        return dict(loss=float(L.detach()), grads=grads, total_norm=total)

    def step_dp(self, x, c, eps_mu, eps_nu, beta, n_total, allreduce):
        """The engine's data-parallel step (mm-vae_amd/csrc/capi.hip mmvae_run): this rank's
        rows with the loss divided by the global batch n_total, backward, SUM all-reduce of
        the registered gradients (``allreduce(list_of_tensors)`` sums in place across ranks),
        then clip_grad_norm_ + Adam on the identical summed gradients of every rank."""
        y = self.m.forward(x, c, eps_mu, eps_nu, True)
        L = loss(x, y, beta, n_total=n_total)
        self.adam.zero_grad()
        L.backward()
        gl = [v.grad for v in self.m.p.values()]
        allreduce(gl)
        grads = OrderedDict((k, v.grad.detach().clone()) for k, v in self.m.p.items())
        total = clip_grad_norm_(gl, self.grad_clip)
        self.adam.step()
        return dict(loss=float(L.detach()), grads=grads, total_norm=total)

    @torch.no_grad()
    def eval_loss(self, x, c, eps_mu, eps_nu, beta):
        """Q12: the reported per-batch loss is a train-mode forward (fresh eps), no update."""
        y = self.m.forward(x, c, eps_mu, eps_nu, True)
        return float(loss(x, y, beta))

    @torch.no_grad()
    def encode(self, x):
        """Recorder path nb.hh:619-657 -> encode_mu(x) without covariate."""
        return self.m.encode_mu(x, None)

    def params(self):
        return OrderedDict((k, v.detach().clone()) for k, v in self.m.p.items())
