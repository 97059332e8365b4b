#!/bin/bash
# The three-waves-per-SIMD pass B (MMVAE_DEC3=1): its parity tests, then x3 headline benches
# without / with it.  Usage: bash tools/ab_dec3.sh TAG [steps]
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
TAG=${1:-d3}; ST=${2:-300}
timeout -k 10 500 python -u -m pytest tests/test_gpu_dec3.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$TAG.test.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG.test.log; [ $rc -eq 0 ] || exit $rc
for spec in base MMVAE_DEC3=1 base MMVAE_DEC3=1; do
  if [ "$spec" == base ]; then envs=""; else envs="$spec"; fi
  env $envs timeout -k 10 200 python bench.py --no-extras --no-cpu --dtype bf16x3 --steps $ST > gpurun_out/$TAG.json 2>gpurun_out/$TAG.err || { tail -3 gpurun_out/$TAG.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/$TAG.json'));print('$spec', round(d['value']), d['ms_per_step'], {k: round(v*1e3,1) for k, v in d['kernel_ms'].items()})"
done
