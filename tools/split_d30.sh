#!/bin/bash
# Pass-B gene-split sweep at the configs[3] shape (D = 30k): one short bench per MMVAE_NSPLIT_D.
mkdir -p gpurun_out
for s in "$@"; do
  MMVAE_NSPLIT_D=$s timeout -k 10 200 python bench.py --no-cpu --genes 30000 --cells 200000 --steps 20 --warmup 3 > gpurun_out/sd_$s.json 2> gpurun_out/sd_$s.err || exit 1
  python3 -c "import json,sys; j=json.load(open('gpurun_out/sd_$s.json')); print('nsD=$s', j['value'], {k: round(v*1e3,1) for k,v in j['kernel_ms'].items() if k.startswith('k_dec')})"
done
