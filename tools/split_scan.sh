#!/bin/bash
# Gene-split occupancy scan (diagnostic): one short bench per MMVAE_NSPLIT_{E,D,A} setting.
# Usage: bash tools/split_scan.sh MODEL SETTING...   e.g. bash tools/split_scan.sh nb X=0 MMVAE_NSPLIT_E=12
MODEL=$1; shift
mkdir -p gpurun_out; out=gpurun_out/split_scan_$MODEL.txt; : > $out
for s in "$@"; do
  env $s timeout -k 10 120 python bench.py --no-cpu --model $MODEL --steps 10 --warmup 3 > gpurun_out/ss.json 2> gpurun_out/ss.err || { tail -3 gpurun_out/ss.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/ss.json')); k=j['kernel_ms']; print(sys.argv[1], 'step', j['ms_per_step'], {n: v for n, v in k.items() if v > 0.02})" "$s" >> $out
done
cat $out
