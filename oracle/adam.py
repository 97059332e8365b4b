"""LibTorch C++ optimiser semantics used by the reference's train loop (test infrastructure).

Reference call sites: ``include/mmvae_alg.hh:234-236`` builds
``torch::optim::Adam(model->parameters(), AdamOptions(lr).weight_decay(1e-4))`` and every
bootstrap step (``mmvae_alg.hh:306-310``) runs ``zero_grad(); loss.backward();
clip_grad_norm_(model->parameters(), grad_clip); adam.step();``.

The algorithms live in LibTorch (third-party, not under /root/reference).  Version pinned:
LibTorch 2.10.0 — ``torch/nn/utils/clip_grad.h:22-92`` (header shipped in this image) and
``torch/csrc/api/src/optim/adam.cpp`` (C++ Adam: L2 weight decay added to the gradient
*after* clipping, ``exp_avg.mul_(b1).add_(g, 1-b1)``, ``exp_avg_sq.mul_(b2).addcmul_(g, g,
1-b2)``, ``denom = sqrt(exp_avg_sq)/sqrt(bc2) + eps``, ``p.addcdiv_(exp_avg, denom,
-lr/bc1)``).  Python's ``torch.optim.Adam`` uses ``lerp_`` and a different op order, so it is
NOT used here.
"""
import math
import torch


def clip_grad_norm_(grads, max_norm):
    """torch::nn::utils::clip_grad_norm_ (LibTorch 2.10 clip_grad.h:54-86), norm_type=2.

    total = ||stack([||g_i||_2])||_2 ; coef = clamp(max_norm/(total+1e-6), max=1);
    every grad is multiplied by coef (always, even when coef == 1).  Returns total (float).
    """
    norms = [g.norm(2) for g in grads]
    total = norms[0] if len(norms) == 1 else torch.stack(norms).norm(2)
    coef = max_norm / (total + 1e-6)
    coef = torch.clamp(coef, max=1.0)
    for g in grads:
        g.mul_(coef)
    return float(total)


class LibTorchAdam:
    """torch::optim::Adam step with AdamOptions(lr).weight_decay(wd), betas (0.9, 0.999), eps 1e-8."""

    def __init__(self, params, lr=1e-3, weight_decay=1e-4, betas=(0.9, 0.999), eps=1e-8):
        self.params = params  # list of leaf tensors (registered parameters, LibTorch order)
        self.lr = lr
        self.wd = weight_decay
        self.b1, self.b2 = betas
        self.eps = eps
        self.state = [None] * len(params)

    @torch.no_grad()
    def step(self):
        for i, p in enumerate(self.params):
            if p.grad is None:
                continue
            grad = p.grad
            if self.state[i] is None:
                self.state[i] = {"step": 0, "exp_avg": torch.zeros_like(p), "exp_avg_sq": torch.zeros_like(p)}
            st = self.state[i]
            st["step"] += 1
            bc1 = 1 - self.b1 ** st["step"]
            bc2 = 1 - self.b2 ** st["step"]
            if self.wd != 0:
                grad = grad.add(p, alpha=self.wd)
            st["exp_avg"].mul_(self.b1).add_(grad, alpha=1 - self.b1)
            st["exp_avg_sq"].mul_(self.b2).addcmul_(grad, grad, value=1 - self.b2)
            denom = (st["exp_avg_sq"].sqrt() / math.sqrt(bc2)).add_(self.eps)
            step_size = self.lr / bc1
            p.addcdiv_(st["exp_avg"], denom, value=-step_size)

    def zero_grad(self):
        # LibTorch 2.x Optimizer::zero_grad(set_to_none=true)
        for p in self.params:
            p.grad = None
