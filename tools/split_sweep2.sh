#!/bin/bash
# x3 headline under split overrides: "VAR=value" specs on the command line (one bench each)
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for spec in base "$@"; do
  if [ "$spec" == base ]; then envs=""; else envs="$spec"; fi
  env $envs timeout -k 10 200 python bench.py --no-extras --no-cpu --dtype ${DT:-bf16x3} --steps 200 ${BENCH_ARGS:-} > gpurun_out/sw.json 2>gpurun_out/sw.err || { tail -3 gpurun_out/sw.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sw.json'));print('$spec', round(d['value']), d['ms_per_step'], {k: round(v*1e3,1) for k, v in d['kernel_ms'].items() if k in ('k_dec_nb','k_dec_lse','k_dec_tail','k_enc_fwd','k_enc_bwd','k_grad_genes','k_latent_bwd','k_latent_fwd')})"
done
