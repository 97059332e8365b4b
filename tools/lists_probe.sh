#!/bin/bash
# k_batch_lists phase ablations (diagnostic build, outputs invalid): MMVAE_DBG 512 = index phase
# only, 8192 = no stream-out, 4096 = no raw-count dots.  Usage: bash tools/lists_probe.sh TAG
TAG=${1:-lp}; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for dbg in 0 512 8192 4096 12288; do
  MMVAE_DBG=$dbg MMVAE_LIB=mm-vae_amd/lib_diag/libmmvae.so timeout -k 10 200 python bench.py --no-extras --no-cpu --steps 100 --warmup 10 > gpurun_out/$TAG.json 2>gpurun_out/$TAG.err || { tail -3 gpurun_out/$TAG.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/$TAG.json'));print('dbg $dbg', {k: round(v*1e3,1) for k, v in d['kernel_ms'].items() if k in ('k_batch_lists','k_prep','k_latent_fwd','k_latent_bwd','k_grad_genes','k_adam')})"
done
