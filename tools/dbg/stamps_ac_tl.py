# pass A timeline (entry / loop / end per wave) for the split given by MMVAE_NSPLIT_A
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "mm-vae_amd", "py"))
os.environ["MMVAE_DBG"] = "256"
import mmvae_amd
B, D, K = 4096, 20000, 64
eng = mmvae_amd.Engine(D=D, K=K, max_batch=B, dtype=os.environ.get("DTYPE", "bf16"), seed=1)
eng.synth_csr(100000, lib_size=2000.0, seed=3)
eng.init_params(seed=7)
for i in range(2):
    eng.eval_loss(np.arange(B), 1.0, step_id=i)
nsa = eng.tiling()["split_ac"]
nwg = (B // 128) * nsa
buf = np.zeros(nwg * 4 * 8, np.float32)
assert mmvae_amd.lib().mmvae_debug_copy(eng._h, 2, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), buf.size) == 0
f = buf.reshape(-1, 8).astype(np.float64)
M = 2 ** 24
t = ((f[:, 3:6] - f[:, 3].min() + M / 2) % M) - M / 2
t -= t[:, 0].min()
ent, ls, le = t[:, 0] / 100, t[:, 1] / 100, t[:, 2] / 100
print("nsA", nsa, "waves", len(t), "span %.1f us" % le.max(), "late starters (>2us)", int((ent > 2).sum()),
      "loop med %.1f us" % np.median(le - ls), "prologue med %.2f" % np.median(ls - ent))
