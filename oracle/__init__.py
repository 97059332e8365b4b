"""oracle/ — CPU restatement of the reference's hot path. TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import anything from here, and only as the *checker* (or the timed CPU baseline), never as
the product path.  The product path is the HIP library ``mm-vae_amd/lib/libmmvae.so``
behind ``include/mmvae_capi.h``; it fails loudly when that library is missing.

Contents
--------
fastmath.py     Bit-exact restatement of P. Mineiro's ``fasterlog``/``fasterlgamma``
                (reference ``include/utils/fastlog.h:75-85``, ``fastgamma.h:58-60``).
adam.py         LibTorch C++ ``torch::optim::Adam::step`` (weight-decay=L2) and
                ``torch::nn::utils::clip_grad_norm_`` semantics
                (reference call sites ``include/mmvae_alg.hh:234-236,306-310``).
nb_oracle.py    NB-VAE forward / loss / backward (LibTorch autograd) — restates
                ``include/models/nb.hh:299-548`` op for op on ATen CPU fp32.
vmf_oracle.py   vMF-VAE — restates ``include/models/vmf.hh:250-440``,
                ``include/operators.hh:13-101`` and ``include/modules/angular.hh:34-70``.
nb_analytic.py  float64 numpy restatement of the *analytic* gradients the HIP kernels
                implement (sparse encoder split, three-pass softmax/NB epilogue).  Used by
                CPU tests to prove the algebra equals autograd before it runs on a GPU.
ref_nb.py       Driver of the reference's own NB model (oracle/_ref/ref_nb_harness, built
                from /root/reference by ``make -C oracle``); writes the NB golden fixtures.
synth.py        Seeded synthetic count-matrix generator (SURVEY §8(d) distribution).

Parity pinning
--------------
NB is pinned to the reference itself.  ``make -C oracle`` compiles the reference's own
model, ``include/models/nb.hh:1-563`` (options, ``nbvae_tImpl``, ``nllik_loss``,
``kl_loss``, ``loss``; the Eigen-based recorder at :564-662 is left out, no stand-in
header), with its ``util.hh`` / ``check.hh`` / ``std_util.hh`` / ``angular.hh`` against
this image's LibTorch 2.10 into ``oracle/_ref/ref_nb_harness`` (``ref_nb_harness.cc``,
driven by ``ref_nb.py``).  It runs the reference's step (``mmvae_alg.hh:234-236,290-310``:
index_select, forward, loss, zero_grad, backward, ``clip_grad_norm_``, Adam) and recovers
the noise its ``randn_like`` drew by the SURVEY Appendix-A re-seed (checked bit-exact).
Every NB golden fixture is that harness's output; ``tests/test_oracle.py`` re-runs the
reference on each fixture (bit-identical) and checks that ``nb_oracle.py`` reproduces the
reference's loss, gradients, clip norm, post-Adam parameters, eval loss and encoder
outputs bit for bit.
vMF is pinned only through its fast-math scalars: ``include/models/vmf.hh:2`` includes
``operators.hh``, whose ``:45`` calls ``SavedVariable::reset_grad_function``, removed in
LibTorch 2.10, so the reference's vMF model does not build here without a source shim.
``fasterlog`` / ``fasterlgamma`` are compiled from the reference's ``fastlog.h`` /
``fastgamma.h`` into ``oracle/_ref/libref_fastmath.so`` and checked bit-exact; the vMF
ELBO restatement runs the reference's op sequence on the same ATen 2.10 kernels.
"""
