"""Diagnostic: bench.py's loader leg alone (20k cells of the synthetic 1M x 20k dataset)."""
import os, sys, json
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "mm-vae_amd", "py"))
import bench
import mmvae_amd
eng, nnz = bench.make_engine(mmvae_amd, "nb", 20000, 64, 4096, "bf16", 100000, 2000.0, 0)
for _ in range(3):
    print(json.dumps(bench.loader_rate(eng, 20000)))
