"""Bit-identity of an env knob: run this twice (with / without the knob) and compare the dumps.
   python tools/bitcheck.py OUT.npz [dtype]   ->  losses, norms, params and grads after 6 steps."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mm-vae_amd", "py"))
import mmvae_amd
out, dt = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "bf16x3")
D, K, B, N = 20000, 64, 4096, 30000
eng = mmvae_amd.Engine(D=D, K=K, max_batch=B, dtype=dt, seed=1)
eng.synth_csr(N, lib_size=2000.0, seed=3)
eng.init_params(seed=7)
eng.graph(True)
res = {}
rng = np.random.default_rng(2)
for s in range(6):
    b = B if s != 3 else B - 200
    cells = rng.integers(0, N, b)
    if s == 2:
        res["eval"] = np.float32(eng.eval_loss(cells, 0.9, step_id=s))
        continue
    l, n = eng.step(cells, 0.9, step_id=s)
    res[f"loss{s}"], res[f"norm{s}"] = np.float32(l), np.float64(n)
for k, v in eng.params(registered_only=True).items():
    res["p/" + k] = v
for k, v in eng.grads().items():
    res["g/" + k] = v
np.savez(out, **res)
if len(sys.argv) > 3:  # compare with a previous dump
    ref = np.load(sys.argv[3])
    bad = [k for k in res if not np.array_equal(ref[k], res[k])]
    print("bit-identical" if not bad else f"DIFFER: {bad[:8]}")
    sys.exit(1 if bad else 0)
