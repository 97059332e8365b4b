#!/bin/bash
# A/B of an environment switch on the quick headline benches (no tests).
# Usage: VAR=MMVAE_NO_SIDE bash tools/ab.sh TAG
TAG=${1:-ab}; VAR=${VAR:-MMVAE_NO_SIDE}
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for dt in ${DTYPES:-bf16x3 bf16}; do
  for v in 0 1; do
    env $VAR=$v timeout -k 10 300 python bench.py --no-extras --no-cpu --dtype $dt --steps ${STEPS:-300} ${BENCH_ARGS:-} > gpurun_out/${TAG}_${dt}_$v.json 2>gpurun_out/${TAG}_${dt}_$v.err || { tail gpurun_out/${TAG}_${dt}_$v.err; exit 2; }
    python -c "import json;d=json.load(open('gpurun_out/${TAG}_${dt}_$v.json'));print('$dt $VAR=$v', round(d['value']), d['ms_per_step'], d.get('median_ms_per_step_synced'))"
  done
done
