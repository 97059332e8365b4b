import sys, numpy as np
sys.path.insert(0, "mm-vae_amd/py"); sys.path.insert(0, "tests")
from test_gpu_graph import _engine
D, K, B = 3000, 32, 256
rng = np.random.default_rng(0)
seq = []
for i in range(4):
    seq.append(rng.integers(0, 3000, B))
seq.append(rng.integers(0, 3000, 100))
for i in range(3):
    seq.append(rng.integers(0, 3000, B))
res = []
for rep in range(4):
    eng = _engine("nb", D, K, B, "f32", False)
    gs = []
    for i, cells in enumerate(seq):
        out = eng.step(cells, 1.0, step_id=100 + i)
        gs.append((out, eng.grads(), eng.params()))
    res.append(gs)
for i in range(len(seq)):
    bad = []
    for k in res[0][i][1]:
        d = [float(np.abs(res[0][i][1][k] - r[i][1][k]).max()) for r in res[1:]]
        if max(d) > 0:
            bad.append((k, d))
    pb = [k for k in res[0][i][2] if any(not np.array_equal(res[0][i][2][k], r[i][2][k]) for r in res[1:])]
    print(i, seq[i].size, [r[i][0] for r in res], "grad diffs:", bad[:4], "param diffs:", pb[:4])
