#!/bin/bash
# Kernel ablation timings (diagnostic): one short bench per MMVAE_DBG value.
# Usage: bash tools/ablate.sh KERNELS BITS...   e.g. bash tools/ablate.sh k_enc_bwd,k_dec_nb 0 1 2 4
ks=$1; shift
mkdir -p gpurun_out
out=gpurun_out/ablate.txt
: > $out
for f in "$@"; do
  MMVAE_DBG=$f timeout -k 10 120 python bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/abl_$f.json 2> gpurun_out/abl_$f.err || exit 1
  python3 - "$f" "$ks" >> $out <<'PY'
import json, sys
f, ks = sys.argv[1], sys.argv[2].split(",")
j = json.load(open(f"gpurun_out/abl_{f}.json"))
print(f"dbg={f}", {k: j["kernel_ms"].get(k) for k in ks}, "step", j["ms_per_step"])
PY
done
cat $out
