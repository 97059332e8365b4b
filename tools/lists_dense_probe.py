"""Dense-row list probe: the same step on one engine config run twice, and under MMVAE_LISTS_PK=0 /
MMVAE_LISTS_XM=1 (each in a fresh process), keys whose gradients differ.  Usage:
python tools/lists_dense_probe.py [nb|vmf] [lib_size]  (prints one JSON line per variant)"""
import json, os, subprocess, sys
import numpy as np

model = sys.argv[1] if len(sys.argv) > 1 else "nb"
lib = float(sys.argv[2]) if len(sys.argv) > 2 else 40000.0
if os.environ.get("_PROBE_CHILD"):
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mm-vae_amd", "py"))
    from mmvae_amd import MODEL_NB, MODEL_VMF, Engine
    D, K, B, N = 20000, 64 if model == "nb" else 32, 256, 600
    eng = Engine(D=D, K=K, max_batch=B, dtype="bf16x3", model=MODEL_VMF if model == "vmf" else MODEL_NB, seed=3)
    nnz = eng.synth_csr(N, lib_size=lib, seed=5)
    eng.init_params(seed=5)
    if os.environ.get("_PROBE_POISON"):
        eng.poison(int(os.environ["_PROBE_POISON"], 16))
    steps = int(os.environ.get("_PROBE_STEPS", "1"))
    out = {}
    for t in range(steps):
        cells = (np.arange(B, dtype=np.int64) * (3 + 2 * t) + 1) % N
        loss, norm = eng.step(cells, 0.7, step_id=t)
        out.update({f"s{t}/{k}": v for k, v in eng.grads().items()})
        out[f"s{t}/loss"] = np.float32(loss)
    np.savez(os.environ["_PROBE_OUT"], **out)
    print(json.dumps({"nnz_per_row": nnz / N, "loss": loss}))
    sys.exit(0)
res = {}
for tag, env in (("pk", {}), ("pk2", {}), ("nopk", {"MMVAE_LISTS_PK": "0"}), ("xm", {"MMVAE_LISTS_XM": "1"}),
                 ("pk_p00", {"_PROBE_POISON": "00"}), ("pk_pFF", {"_PROBE_POISON": "FF"}), ("nopk_pFF", {"MMVAE_LISTS_PK": "0", "_PROBE_POISON": "FF"})):
    out = f"/tmp/_probe_{tag}.npz"
    e = dict(os.environ, _PROBE_CHILD="1", _PROBE_OUT=out, **env)
    subprocess.run([sys.executable, __file__, model, str(lib)], env=e, check=True)
    res[tag] = dict(np.load(out))
for tag in ("pk2", "nopk", "xm", "pk_p00", "pk_pFF", "nopk_pFF"):
    diff = {k: float(np.abs(res[tag][k] - res["pk"][k]).max()) for k in res["pk"] if not np.array_equal(res[tag][k], res["pk"][k])}
    print(json.dumps({"vs_pk": tag, "differing": diff}))
