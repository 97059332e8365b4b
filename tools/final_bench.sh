#!/bin/bash
# The driver's default bench (NB headline, every line, CPU baseline) and the vMF headline bench.
# Usage: bash tools/final_bench.sh TAG
TAG=${1:-fb}; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 400 python bench.py > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err || { tail gpurun_out/$TAG.bench.err; exit 2; }
timeout -k 10 300 python bench.py --model vmf > gpurun_out/$TAG.bench_vmf.json 2> gpurun_out/$TAG.bench_vmf.err || { tail gpurun_out/$TAG.bench_vmf.err; exit 3; }
python -c "import json;d=json.load(open('gpurun_out/$TAG.bench.json'));print(d['value'], d['ms_per_step'], [(l['label'][:40], l['value']) for l in d['lines']])"
