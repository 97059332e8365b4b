#!/bin/bash
# A/B of an env knob: NB parity tests under the knob, then headline benches without / with it.
# Usage: bash tools/ab_env.sh TAG "VAR=value [VAR2=value]" [dtypes]
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
TAG=$1; KNOB=$2; DTS=${3:-"bf16x3 bf16"}
env $KNOB timeout -k 10 400 python -u -m pytest tests/test_gpu_nb.py tests/test_gpu_tiling.py tests/test_gpu_graph.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG.test.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG.test.log; [ $rc -eq 0 ] || exit $rc
for dt in $DTS; do
for spec in base "$KNOB"; do
  if [ "$spec" == base ]; then envs=""; else envs="$spec"; fi
  env $envs timeout -k 10 200 python bench.py --no-extras --no-cpu --dtype $dt --steps 300 > gpurun_out/$TAG.json 2>gpurun_out/$TAG.err || { tail -3 gpurun_out/$TAG.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/$TAG.json'));print('$dt', '$spec', round(d['value']), d['ms_per_step'], {k: round(v*1e3,1) for k, v in d['kernel_ms'].items()})"
done; done
