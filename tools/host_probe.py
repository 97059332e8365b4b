"""Host cost of one step launch vs the GPU step, graph and eager (diagnostic).

    python tools/host_probe.py
Prints, per mode: (1) host microseconds per mmvae_run call at B = 4096 on a 64-gene dataset, where
the GPU step is short, so the call is host-bound; (2) ms/step of the headline shape, alternating
graph / eager twice on the same engine."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import mmvae_amd  # noqa: E402
import torch  # noqa: E402


def per_call(eng, batches, n):
    for s in range(20):
        eng.run(batches[s % len(batches)], 1.0, update=True, step_id=s, sync=False)
    eng.sync()
    t0 = time.perf_counter()
    for s in range(n):
        eng.run(batches[s % len(batches)], 1.0, update=True, step_id=100 + s, sync=False)
    t1 = time.perf_counter()
    eng.sync()
    t2 = time.perf_counter()
    return (t1 - t0) / n * 1e6, (t2 - t0) / n * 1e6


B = 4096
batches = [mmvae_amd.shard_batch(s, B, 1000000, 0, 1)[0] for s in range(64)]
if not os.environ.get("HP_BENCH_ONLY"):  # HP_BENCH_ONLY=1: the headline shape only
    small, _ = bench.make_engine(mmvae_amd, "nb", 64, 64, B, "bf16x3", 1000000, 30.0, 0)
    for g in (True, False, True, False):
        small.graph(g)
        h, w = per_call(small, batches, 500)
        print(f"D=64    graph={g!s:5s} host us/call {h:7.1f}  wall us/step {w:7.1f}", flush=True)
    del small
    torch.cuda.synchronize()
eng, _ = bench.make_engine(mmvae_amd, "nb", 20000, 64, B, "bf16x3", 1000000, 2000.0, 0)
for g in (True, False, True, False):
    eng.graph(g)
    h, w = per_call(eng, batches, 1000)
    print(f"D=20000 graph={g!s:5s} host us/call {h:7.1f}  wall us/step {w:7.1f}", flush=True)
