#!/bin/bash
# vMF decoder sweep: builds (tools/build_variant.sh NAME, "base" = lib/) x decoder splits.
# Usage: bash tools/vmf_sweep.sh TAG "base NAME.." "12 16" [dtype]
TAG=$1; LIBS=$2; SPLITS=$3; DT=${4:-bf16x3}
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for v in $LIBS; do for ns in $SPLITS; do
  envs="MMVAE_NSPLIT_D=$ns"; [ $v == base ] || envs="$envs MMVAE_LIB=mm-vae_amd/lib_$v/libmmvae.so"
  env $envs timeout -k 10 200 python bench.py --model vmf --no-extras --no-cpu --dtype $DT --steps ${STEPS:-300} > gpurun_out/${TAG}.json 2>gpurun_out/${TAG}.err || { tail -3 gpurun_out/${TAG}.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}.json'));print('$v ns=$ns $DT', round(d['value']), d['ms_per_step'], {k: round(v*1e3,1) for k, v in d['kernel_ms'].items() if k.startswith(('k_vdec','k_enc'))})"
done; done
