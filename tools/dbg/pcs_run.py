"""Diagnostic: a few NB steps at the configs[1] shape (target of rocprofv3 PC sampling)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "mm-vae_amd", "py"))
import mmvae_amd
B, D, K = 4096, 20000, 64
eng = mmvae_amd.Engine(D=D, K=K, max_batch=B, dtype=os.environ.get("DTYPE", "bf16"), seed=1)
eng.synth_csr(100000, lib_size=2000.0, seed=3)
eng.init_params(seed=7)
for i in range(int(os.environ.get("STEPS", "20"))):
    eng.step((np.arange(B) + i * B) % 100000, 1.0, step_id=i)
eng.sync()
print("done")
