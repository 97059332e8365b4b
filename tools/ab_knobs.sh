#!/bin/bash
# Headline x3 benches under several env settings (no parity run): bash tools/ab_knobs.sh TAG STEPS "SPEC1" "SPEC2" ...
# (SPEC: "base" or "VAR=value [VAR2=value]")
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
TAG=$1; ST=$2; shift 2
for spec in "$@"; do
  if [ "$spec" == base ]; then envs=""; else envs="$spec"; fi
  env $envs timeout -k 10 200 python bench.py --no-extras --no-cpu --dtype ${DT:-bf16x3} --steps $ST > gpurun_out/$TAG.json 2>gpurun_out/$TAG.err || { tail -3 gpurun_out/$TAG.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/$TAG.json'));print('$spec', round(d['value']), d['ms_per_step'], {k: round(v*1e3,1) for k, v in d['kernel_ms'].items()})"
done
