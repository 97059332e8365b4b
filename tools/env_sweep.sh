#!/bin/bash
# Headline bench under each environment setting.  Usage: bash tools/env_sweep.sh TAG MODEL DTYPE "ENV1=a ENV2=b" "ENV1=c" ...
TAG=$1; M=$2; DT=$3; shift 3
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for spec in "base" "$@"; do
  envs=""; [ "$spec" == base ] || envs="$spec"
  env $envs timeout -k 10 200 python bench.py --model $M --no-extras --no-cpu --dtype $DT --steps ${STEPS:-300} > gpurun_out/$TAG.json 2>gpurun_out/$TAG.err || { tail -3 gpurun_out/$TAG.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/$TAG.json'));print('$spec', round(d['value']), d['ms_per_step'], {k: round(v*1e3,1) for k, v in d['kernel_ms'].items()})"
done
