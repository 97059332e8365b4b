"""Diagnostic: realtime phase timeline of k_latent_bwd (KER=bwd, MMVAE_DBG=1024) or k_latent_fwd (KER=fwd, 2048)."""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mm-vae_amd", "py"))
KER = os.environ.get("KER", "bwd")
os.environ["MMVAE_DBG"] = str((1024 if KER == "bwd" else 2048) | int(os.environ.get("EXTRA", "0")))
import mmvae_amd
B, D, K = 4096, 20000, 64
eng = mmvae_amd.Engine(D=D, K=K, max_batch=B, dtype=os.environ.get("DTYPE", "bf16x3"), seed=1)
eng.synth_csr(100000, lib_size=2000.0, seed=3)
eng.init_params(seed=7)
for i in range(3):  # fwd: eval path (pass C, which also writes slabC, does not run)
    if KER == "bwd":
        eng.step(np.arange(B), 1.0, step_id=i)
    else:
        eng.eval_loss(np.arange(B), 1.0, step_id=i)
nwg = B // 16
NWV = int(os.environ.get("NWV", "16"))  # waves per latent workgroup (MMVAE_LAT_NW=4: 4)
buf = np.zeros(nwg * NWV * 8, np.float32)
rc = mmvae_amd.lib().mmvae_debug_copy(eng._h, 2, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), buf.size)
assert rc == 0
f = buf.reshape(-1, 8).astype(np.float64)
M = 2 ** 24
ref = f[0, 0]
t = ((f[:, :7] - ref + M / 2) % M) - M / 2
t -= t[:, 0].min()
names = (["loads", "-", "per-cell", "dh MFMA+stores", "dW MFMA", "small+drain"] if KER == "bwd" else
         ["loads", "rowx+mvec", "heads MFMA", "per-cell", "kl+drain", "-"])
ph = np.diff(t, axis=1) / 100.0
print("kernel span %.2f us; wave start spread %.2f us" % (t[:, 6].max() / 100, t[:, 0].max() / 100))
for n, v in zip(names, ph.mean(0)):
    print("  %-16s %6.2f us" % (n, v))
