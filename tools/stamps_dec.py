"""Diagnostic: per-phase cycle shares of k_dec_nb's tile loop (MMVAE_DBG=64 stamp build)."""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mm-vae_amd", "py"))
os.environ["MMVAE_DBG"] = "64"
import mmvae_amd
B, D, K = 4096, 20000, 64
eng = mmvae_amd.Engine(D=D, K=K, max_batch=B, dtype=os.environ.get("DTYPE", "bf16"), seed=1)
eng.synth_csr(100000, lib_size=2000.0, seed=3)
eng.init_params(seed=7)
for i in range(3):  # UPDATE=1: the training instance (outputs invalid under stamps), else the eval one
    if os.environ.get("UPDATE") == "1":
        eng.step(np.arange(B), 1.0, step_id=i)
    else:
        eng.eval_loss(np.arange(B), 1.0, step_id=i)
nsd = int(os.environ.get("NSD", "8"))
NW = int(os.environ.get("NW", "8"))  # waves per pass-B workgroup (DEC_NW; 4 for MMVAE_DEC3=1)
nwg = (B // (16 * NW)) * nsd
buf = np.zeros(nwg * NW * 16, np.float32)
rc = mmvae_amd.lib().mmvae_debug_copy(eng._h, 1, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), buf.size)
assert rc == 0
full = buf.reshape(-1, 16)
np.save(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "stamps_dec.npy"), full)
st = full[:, :7]
names = ["logits+exp", "sparse", "fetch", "epilogue", "dz+zero", "barrier+slab", "stage+barrier"]
tot = st.sum(1)
ntile = (313 + nsd - 1) // nsd
print("waves", st.shape[0], "mean total cycles/wave %.0f (%.0f per tile)" % (tot.mean(), tot.mean() / ntile))
for n, v in zip(names, st.mean(0)):
    print("  %-14s %8.0f cyc/wave  %6.0f per tile  %5.1f%%" % (n, v, v / ntile, 100 * v / tot.mean()))
print("max-wave total / mean: %.3f" % (tot.max() / tot.mean()))
# imbalance: per-wave totals by gene split and by row block (blockIdx = rb * nsD + sp)
tw = tot.reshape(-1, NW)           # [wg][wave]
wg = tw.max(1)                     # a workgroup ends with its slowest wave
sp = np.arange(wg.size) % nsd
rb = np.arange(wg.size) // nsd
print("per split (mean of wg max, k cycles):", [round(float(wg[sp == s].mean()) / 1e3, 1) for s in range(nsd)])
rbm = np.array([wg[rb == r].mean() for r in range(rb.max() + 1)])
print("row blocks: min %.1f mean %.1f max %.1f (k cycles)" % (rbm.min() / 1e3, rbm.mean() / 1e3, rbm.max() / 1e3))
print("wave spread inside a workgroup (max/min): %.3f" % float((tw.max(1) / tw.min(1)).mean()))
