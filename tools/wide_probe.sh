#!/bin/bash
# Kernel trace of the wide path (NB 100k x 20k, --mean_latent 128): per-dispatch rows for the
# GEMM shapes.   Usage: bash tools/wide_probe.sh TAG [DTYPE]
TAG=${1:-wide}; DT=${2:-f32}
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_trace -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu --no-extras --latent 128 --cells 100000 --dtype $DT --steps 10 --warmup 3 --kernel-steps 1 \
  > $R/gpurun_out/${TAG}.json 2> $R/gpurun_out/${TAG}.err || { tail -5 $R/gpurun_out/${TAG}.err; exit 1; }
python3 -c "import json;d=json.load(open('$R/gpurun_out/${TAG}.json'));print(d['value'], d['ms_per_step'])"
