#!/bin/bash
# A/B of an alternative build (tools/build_variant.sh NAME) on the quick headline benches.
# Usage: bash tools/ab_lib.sh TAG NAME [models] [dtypes]   (NAME "-": the in-tree build only)
TAG=$1; NAME=$2; MODELS=${3:-"nb vmf"}; DTS=${4:-"bf16x3"}
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for m in $MODELS; do for dt in $DTS; do for v in base ${NAME/#-/}; do
  if [ $v == base ]; then envs=""; else envs="MMVAE_LIB=mm-vae_amd/lib_$v/libmmvae.so"; fi
  env $envs timeout -k 10 200 python bench.py --model $m --no-extras --no-cpu --dtype $dt --steps ${STEPS:-300} > gpurun_out/${TAG}.json 2>gpurun_out/${TAG}.err || { tail -3 gpurun_out/${TAG}.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}.json'));print('$m $dt $v', round(d['value']), d['ms_per_step'], {k: round(v*1e3,1) for k, v in d['kernel_ms'].items() if k.startswith(tuple('${KF:-k_dec k_vdec k_enc}'.split()))})"
done; done; done
