"""Does a host->device copy on the DMA engines slow the step's kernels the way the zero-copy
gather does?  Per-kernel times of the resident NB x3 step (100k x 20k) alone and
with 27 MB hipMemcpyAsync copies from pinned memory queued on a side stream."""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mm-vae_amd", "py"))
import numpy as np
import torch
torch.cuda.set_device(0)
import bench
import mmvae_amd
B, cells = 4096, 100000
eng, nnz = bench.make_engine(mmvae_amd, "nb", 20000, 64, B, "bf16x3", cells, 2000.0, 0)
batches = [(s * B + np.arange(B)) % cells for s in range(60)]
nb = int(4 * nnz / cells * B)
h = torch.empty(nb // 4, dtype=torch.int32, pin_memory=True)
d = torch.empty(nb // 4, dtype=torch.int32, device="cuda")
side = torch.cuda.Stream()
def run(copies):
    bench.time_steps(eng, batches, 1.0, B, 0, 10, 5)
    if copies:
        with torch.cuda.stream(side):
            for _ in range(copies):
                d.copy_(h, non_blocking=True)
    t0 = time.perf_counter()
    per, step = bench.kernel_times(eng, batches, 1.0, B, 0, 30)
    t1 = time.perf_counter()
    side.synchronize()
    t2 = time.perf_counter()
    return {"copies": copies, "step_ms": round((t1 - t0) / 30 * 1e3, 4), "copies_done_ms": round((t2 - t0) * 1e3, 2),
            "kernel_us": {k: round(v * 1e3, 1) for k, v in sorted(per.items(), key=lambda kv: -kv[1])[:6]}}
print(json.dumps({"bytes_per_copy": nb, "alone": run(0), "with_dma": run(30)}, indent=1))
