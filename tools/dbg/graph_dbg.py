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
eps = rng.standard_normal(B * (K + 1)).astype(np.float32)
seq.append(("step", rng.integers(0, 3000, B), 0.5, B, 0, eps))
for i in range(3):
    seq.append(("step", rng.integers(0, 3000, B), 1.0, B, 0, None))
res = {}
for name, graph in (("eager", False), ("eager2", False), ("graph", True)):
    eng = _engine("nb", D, K, B, "f32", graph)
    tr = []
    for i, (kind, cells, beta, n_total, ro, ep) in enumerate(seq):
        if kind == "eval":
            tr.append((eng.eval_loss(cells, beta, step_id=100 + i), 0.0))
        else:
            tr.append(eng.step(cells, beta, n_total=n_total, row_offset=ro, step_id=100 + i, eps=ep))
    res[name] = (tr, eng.params())
for i in range(len(seq)):
    print(i, seq[i][0], [res[n][0][i] for n in res])
for k in res["eager"][1]:
    a, b, c = res["eager"][1][k], res["eager2"][1][k], res["graph"][1][k]
    if not (np.array_equal(a, b) and np.array_equal(a, c)):
        print(k, np.abs(a - b).max(), np.abs(a - c).max())
