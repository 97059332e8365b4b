"""Run bench.streamed() alone (the out-of-core line of the default bench)."""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mm-vae_amd", "py"))
import torch
torch.cuda.set_device(0)  # as bench.main: torch's HIP runtime first
import bench
import mmvae_amd
print(json.dumps(bench.streamed(mmvae_amd, "nb", 20000, 64, 4096, "bf16x3", int(os.environ.get("CELLS", "100000")), 2000.0,
                                label="streamed probe")))
