import sys, numpy as np
sys.path.insert(0, "mm-vae_amd/py")
from mmvae_amd import Engine
D, K, B = 30000, 64, 8192
engs = {}
for dtype in ("bf16x3", "bf16", "fp8"):
    eng = Engine(D=D, K=K, max_batch=B, dtype=dtype, seed=3)
    eng.synth_csr(20000, lib_size=2000.0, seed=5)
    eng.init_params(seed=7)
    cells = np.random.default_rng(1).integers(0, 20000, B)
    l0 = eng.eval_loss(cells, 1.0, step_id=4)
    loss, norm = eng.step(cells, 1.0, step_id=4)
    l1 = eng.eval_loss(cells, 1.0, step_id=4)
    print(dtype, repr(l0), repr(loss), repr(norm), repr(l1))
    engs[dtype] = eng  # keep alive
