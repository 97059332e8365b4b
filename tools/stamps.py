"""Diagnostic: per-phase cycle shares of k_enc_fwd's tile loop (MMVAE_DBG=32 stamp build)."""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mm-vae_amd", "py"))
os.environ["MMVAE_DBG"] = "32"
import mmvae_amd
B, D, K = 4096, 20000, 64
eng = mmvae_amd.Engine(D=D, K=K, max_batch=B, dtype=os.environ.get("DTYPE", "bf16"), seed=1)
eng.synth_csr(100000, lib_size=2000.0, seed=3)
eng.init_params(seed=7)
for i in range(3):
    eng.eval_loss(np.arange(B), 1.0, step_id=i)
nse = eng.tiling()["split_enc"]
nwg = (B // 64) * nse
buf = np.zeros(nwg * 4 * 8, np.float32)
rc = mmvae_amd.lib().mmvae_debug_copy(eng._h, 0, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), buf.size)
assert rc == 0
st = buf.reshape(-1, 8)
ntile = eng.tiling()["tps_enc"]
m = st.mean(0)
print("waves", st.shape[0], "per tile: MFMA+wait %.0f  zero+scatter %.0f  fetch+stage %.0f  barrier %.0f" % tuple(m[:4] / ntile))
print("prologue+tail %.0f cycles, wave wall %.0f mean / %.0f max cycles" % (m[4], m[6], st[:, 6].max()))
# balance: per gene split (mean over row blocks of the workgroup's slowest wave) and per row block
wall = st[:, 6].reshape(-1, 4).max(1)          # [wg]
wg_sp = wall.reshape(-1, nse)                   # [rb][sp]
print("per split (k cycles):", np.round(wg_sp.mean(0) / 1e3, 1).tolist())
print("per row block: min %.1f mean %.1f max %.1f (k cycles)" % (wg_sp.max(1).min() / 1e3, wg_sp.max(1).mean() / 1e3, wg_sp.max(1).max() / 1e3))
sc = st[:, 1].reshape(-1, 4).mean(1).reshape(-1, nse)  # zero+scatter cycles per wg
print("scatter per split (k cycles):", np.round(sc.mean(0) / 1e3, 1).tolist())
