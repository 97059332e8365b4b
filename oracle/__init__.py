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
synth.py        Seeded synthetic count-matrix generator (SURVEY §8(d) distribution).

Parity pinning
--------------
The reference's model headers cannot be compiled here: ``include/models/nb.hh`` and
``vmf.hh`` define their recorders on Eigen3 (absent from this image, no network), and the
brief forbids stand-in headers.  The arithmetic of the path lives in the reference's
third-party dependency LibTorch/ATen; this image ships LibTorch 2.10.0 (the same ATen
kernels, via the ``torch`` Python package).  The oracle therefore executes the
reference's own call sequence (file:line cited per function) on ATen 2.10 CPU fp32, and
the two scalar fast-math helpers are pinned bit-exactly against the reference's own
``fastlog.h``/``fastgamma.h`` compiled from ``/root/reference`` into ``oracle/_ref``.
"""
