#!/bin/bash
# One iteration GPU call: full GPU suite, then quick headline benches (x3, bf16) with kernel times.
# Usage: bash tools/iter.sh TAG [skip-tests]
TAG=${1:-it}
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG.test.log 2>&1 || { tail -40 gpurun_out/$TAG.test.log; exit 1; }
  tail -2 gpurun_out/$TAG.test.log
fi
for dt in ${DTYPES:-bf16x3 bf16}; do
  timeout -k 10 300 python bench.py --no-extras --no-cpu --dtype $dt --steps ${STEPS:-200} ${BENCH_ARGS:-} > gpurun_out/${TAG}_$dt.json 2>gpurun_out/${TAG}_$dt.err || { tail gpurun_out/${TAG}_$dt.err; exit 2; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_$dt.json'));print('$dt', round(d['value']), d['ms_per_step'], d['device_ms_per_step'], d.get('median_ms_per_step_synced'));print(d['kernel_ms'])"
done
