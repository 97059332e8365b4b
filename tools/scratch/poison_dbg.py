import sys, numpy as np
sys.path.insert(0, "mm-vae_amd/py")
from mmvae_amd import Engine, MODEL_NB, MODEL_VMF
for model in ("nb", "vmf"):
    for B in (100, 256, 37):
        for poison in (None, 0xFF):
            eng = Engine(D=3000, K=32, max_batch=256, dtype="bf16", seed=9, model=MODEL_VMF if model == "vmf" else MODEL_NB)
            eng.synth_csr(3000, lib_size=1500.0, seed=4)
            eng.init_params(seed=13)
            cells = np.random.default_rng(1).integers(0, 3000, B)
            if poison is not None:
                eng.poison(poison)
            loss, norm = eng.step(cells, 1.0, step_id=3)
            g = eng.grads()
            bad = {k: int(np.sum(~np.isfinite(v))) for k, v in g.items() if not np.all(np.isfinite(v))}
            if poison is None:
                ref = g
                print(model, B, "clean", loss, norm)
            else:
                diff = {k: float(np.abs(v - ref[k]).max()) for k, v in g.items() if np.all(np.isfinite(v)) and not np.array_equal(v, ref[k])}
                print(model, B, "poison", loss, norm, "nonfinite:", bad, "diff:", diff)
