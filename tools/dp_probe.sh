#!/bin/bash
# The DP exchange's fixed cost on one GPU (bench.py dp_exchange): bash tools/dp_probe.sh TAG
TAG=${1:-dp}; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 300 python -c "
import sys, json; sys.argv = ['bench.py']; sys.path.insert(0, 'mm-vae_amd/py')
import torch; torch.cuda.set_device(0)
import bench, mmvae_amd
print(json.dumps(bench.dp_exchange(mmvae_amd, 20000, 64, 4096, 'bf16x3', 1000000, 2000.0)))
" > gpurun_out/$TAG.dp.json 2> gpurun_out/$TAG.dp.err || { tail gpurun_out/$TAG.dp.err; exit 1; }
cat gpurun_out/$TAG.dp.json
