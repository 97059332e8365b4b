"""Diagnostic: per-phase cycles of the vMF decoder passes (k_vdec_fwd / k_vdec_bwd) tile loop.
Needs the -DMMVAE_DIAG build (tools/build_variant.sh diag -DMMVAE_DIAG; MMVAE_LIB points at it)."""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mm-vae_amd", "py"))
os.environ["MMVAE_DBG"] = os.environ.get("DBG", "256")
import mmvae_amd
B, D, K = 4096, 20000, 32
dt = os.environ.get("DT", "bf16x3")
eng = mmvae_amd.Engine(D=D, K=K, max_batch=B, dtype=dt, seed=1, model=mmvae_amd.MODEL_VMF)
eng.synth_csr(100000, lib_size=2000.0, seed=3)
eng.init_params(seed=7)
nsd = int(os.environ.get("MMVAE_NSPLIT_D", "12"))
nsf = int(os.environ.get("MMVAE_NSPLIT_F", "16"))  # the forward pass's own split
names = ["entry fetch", "gene blocks", "barrier 1", "slab store", "stage+barrier 2", "stage load", "zero", "visit"]
for label, run in (("fwd", lambda i: eng.eval_loss(np.arange(B), 1.0, step_id=i)),
                   ("bwd", lambda i: eng.step(np.arange(B), 1.0, step_id=i))):
    for i in range(3):
        run(i)
    nwg = (B // 64) * (nsf if label == "fwd" else nsd)
    buf = np.zeros(nwg * 4 * 12, np.float32)
    rc = mmvae_amd.lib().mmvae_debug_copy(eng._h, 1, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), buf.size)
    assert rc == 0
    full = buf.reshape(-1, 12)
    nt = full[:, 8:9]
    per = full[:, :8] / np.maximum(nt, 1)
    tot = per.sum(1).mean()
    print(label, dt, "waves", full.shape[0], "tiles/wave %.1f" % nt.mean(), "cycles per tile %.0f:" % tot,
          ", ".join("%s %.0f" % (n, v) for n, v in zip(names, per.mean(0))))
