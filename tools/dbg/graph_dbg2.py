import sys, numpy as np
sys.path.insert(0, "mm-vae_amd/py"); sys.path.insert(0, "tests")
from test_gpu_graph import _engine
D, K, B = 3000, 32, 256
rng = np.random.default_rng(0)
seq = []
for i in range(4):
    seq.append(("step", rng.integers(0, 3000, B), 1.0, B, 0, None))
seq.append(("step", rng.integers(0, 3000, 100), 1.0, 100, 0, None))
seq.append(("step", rng.integers(0, 3000, B), 0.5, B, 0, None))
seq.append(("eval", rng.integers(0, 3000, B), 0.5, B, 0, None))
seq.append(("step", rng.integers(0, 3000, B), 0.5, 4 * B, 3 * B, None))
variant = sys.argv[1] if len(sys.argv) > 1 else "full"
if variant == "noeval":
    seq = [s for s in seq if s[0] != "eval"]
if variant == "noragged":
    seq = [s for s in seq if s[1].size == B]
res = []
for rep in range(4):
    eng = _engine("nb", D, K, B, "f32", False)
    for i, (kind, cells, beta, n_total, ro, ep) in enumerate(seq):
        if kind == "eval":
            eng.eval_loss(cells, beta, step_id=100 + i)
        else:
            out = eng.step(cells, beta, n_total=n_total, row_offset=ro, step_id=100 + i, eps=ep)
    res.append((out, eng.grads()))
print(variant, [r[0] for r in res])
for k in res[0][1]:
    d = [float(np.abs(res[0][1][k] - r[1][k]).max()) for r in res[1:]]
    if max(d) > 0:
        i = np.argmax(np.abs(res[0][1][k] - res[1][1][k]).ravel())
        print(k, d, res[0][1][k].shape, "argmax", i)
