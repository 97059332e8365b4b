"""In-process repeatability probe: the same two dense steps on fresh engines created one after the
other in ONE process (default, default again, MMVAE_LISTS_PK=0, default), keys that differ from the
first run.  Usage: python tools/lists_inproc_probe.py [nb|vmf] [lib_size] [B]"""
import json, os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mm-vae_amd", "py"))
from mmvae_amd import MODEL_NB, MODEL_VMF, Engine

model = sys.argv[1] if len(sys.argv) > 1 else "nb"
lib = float(sys.argv[2]) if len(sys.argv) > 2 else 40000.0
B = int(sys.argv[3]) if len(sys.argv) > 3 else 256
D, K, N = 20000, 64 if model == "nb" else 32, 600


def run():
    eng = Engine(D=D, K=K, max_batch=B, dtype="bf16x3", model=MODEL_VMF if model == "vmf" else MODEL_NB, seed=3)
    eng.synth_csr(N, lib_size=lib, seed=5)
    eng.init_params(seed=5)
    out = {}
    for t in range(2):
        cells = (np.arange(B, dtype=np.int64) * (3 + 2 * t) + 1) % N
        loss, _ = eng.step(cells, 0.7, step_id=t)
        out.update({f"s{t}/{k}": v for k, v in eng.grads().items()})
        out[f"s{t}/loss"] = np.float32(loss)
    eng.close()
    return out


res = []
for tag, env in (("a", {}), ("a2", {}), ("nopk", {"MMVAE_LISTS_PK": "0"}), ("a3", {})):
    for k in ("MMVAE_LISTS_PK",):
        os.environ.pop(k, None)
    os.environ.update(env)
    res.append((tag, run()))
base = res[0][1]
for tag, r in res[1:]:
    diff = {k: float(np.abs(r[k] - base[k]).max()) for k in base if not np.array_equal(r[k], base[k])}
    print(json.dumps({"vs_a": tag, "n_differing": len(diff), "differing": dict(list(diff.items())[:6])}))
