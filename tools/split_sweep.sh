#!/bin/bash
# Gene-split sweep (diagnostic): bash tools/split_sweep.sh VAR "bench args" values...
#   e.g. bash tools/split_sweep.sh MMVAE_NSPLIT_A "--genes 20000" 16 32 64
var=$1; args=$2; shift 2
mkdir -p gpurun_out
for s in "$@"; do
  env $var=$s timeout -k 10 200 python bench.py --no-cpu $args --steps 20 --warmup 3 > gpurun_out/sw_$s.json 2> gpurun_out/sw_$s.err || exit 1
  python3 -c "import json; j=json.load(open('gpurun_out/sw_$s.json')); print('$var=$s', j['value'], {k: round(v*1e3,1) for k,v in j['kernel_ms'].items() if k.startswith(('k_dec','k_enc','k_vdec'))})"
done
