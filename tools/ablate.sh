#!/bin/bash
# Pass-B ablation timings (diagnostic): bench per MMVAE_DBG value, k_dec_nb ms.
set -e
out=gpurun_out/ablate.txt
: > $out
for f in "$@"; do
  MMVAE_DBG=$f timeout -k 10 120 python bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/abl_$f.json 2> gpurun_out/abl_$f.err
  python3 -c "import json,sys; j=json.load(open('gpurun_out/abl_$f.json')); print('dbg=$f', j['kernel_ms'])" >> $out
done
cat $out
