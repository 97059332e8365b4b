"""Diagnostic: per-phase cycles of decoder pass A (k_dec_lse) tile loop (MMVAE_DBG=256 stamp build)."""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mm-vae_amd", "py"))
os.environ["MMVAE_DBG"] = "256"
import mmvae_amd
B, D, K = 4096, 20000, 64
eng = mmvae_amd.Engine(D=D, K=K, max_batch=B, dtype=os.environ.get("DT", "bf16x3"), seed=1)
eng.synth_csr(100000, lib_size=2000.0, seed=3)
eng.init_params(seed=7)
for i in range(2):
    eng.eval_loss(np.arange(B), 1.0, step_id=i)   # pass A stamps land in dzp (pass B overwrites? no: B stamps off)
nsa = eng.tiling()["split_ac"]
nwg = (B // 128) * nsa  # 128 rows per workgroup
buf = np.zeros(nwg * 4 * 8, np.float32)
rc = mmvae_amd.lib().mmvae_debug_copy(eng._h, 2, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), buf.size)
assert rc == 0
full = buf.reshape(-1, 8)
np.save(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "stamps_ac.npy"), full)
st = full[:, [7, 0, 1, 2]]
ntile = (313 + nsa - 1) // nsa
print("waves", st.shape[0], "splits", nsa, "per tile cycles: logit MFMA %.0f  element math %.0f  store+barrier %.0f  slab/loop %.0f" % tuple(st.mean(0) / ntile))
