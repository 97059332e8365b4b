"""Diagnostic: per-phase cycles of k_enc_bwd's tile loop (MMVAE_DBG=16384, -DMMVAE_DIAG build)."""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mm-vae_amd", "py"))
os.environ["MMVAE_DBG"] = "16384"
import mmvae_amd
B, D, K = 4096, 20000, 64
eng = mmvae_amd.Engine(D=D, K=K, max_batch=B, dtype=os.environ.get("DTYPE", "bf16x3"), seed=1)
eng.synth_csr(100000, lib_size=2000.0, seed=3)
eng.init_params(seed=7)
for i in range(3):
    eng.step(np.arange(B), 1.0, step_id=i)
nsb = eng.tiling()["split_encb"] if "split_encb" in eng.tiling() else None
n = (B // 64) * 64 * 8  # generous: (row blocks x splits) x 4 waves x 8 floats fits the slab
buf = np.zeros(n * 4, np.float32)
rc = mmvae_amd.lib().mmvae_debug_copy(eng._h, 4, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), buf.size)
assert rc == 0
f = buf.reshape(-1, 8)
f = f[f[:, 6] > 0]  # waves that ran tiles
nt = f[:, 6].mean()
names = ["raw sums", "M + W dot", "barrier 1", "slab + scatter", "fetch + barrier 2"]
print("waves %d, tiles per wave %.1f, tiling %s" % (f.shape[0], nt, eng.tiling()))
for i, nm in enumerate(names):
    print("  %-18s %7.0f cycles per tile" % (nm, (f[:, i] / f[:, 6]).mean()))
print("  wall %.0f cycles mean, %.0f max" % (f[:, 5].mean(), f[:, 5].max()))
