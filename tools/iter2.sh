#!/bin/bash
# Full GPU suite, then quick NB (x3, bf16) and vMF (x3, bf16; 100k cells) benches with kernel times.
TAG=${1:-it}
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG.test.log 2>&1 || { tail -40 gpurun_out/$TAG.test.log; exit 1; }
tail -2 gpurun_out/$TAG.test.log
for m in nb vmf; do for dt in bf16x3 bf16; do
  extra=""; [ $m == vmf ] && extra="--cells 100000"
  timeout -k 10 300 python bench.py --no-extras --no-cpu --model $m --dtype $dt --steps 300 $extra > gpurun_out/${TAG}_${m}_$dt.json 2>gpurun_out/${TAG}.err || { tail gpurun_out/${TAG}.err; exit 2; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_${m}_$dt.json'));print('$m $dt', round(d['value']), d['ms_per_step'], {k: round(v*1e3,1) for k, v in d['kernel_ms'].items()})"
done; done
