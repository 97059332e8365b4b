#!/bin/bash
# Wide path A/B: the wide parity tests, then the K = 128 bench line under a kernel trace once per
# environment setting.   Usage: bash tools/wide_ab.sh TAG DTYPE "ENV1" "ENV2" ...   ("-" = none)
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
TAG=$1; DT=$2; shift 2
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/$TAG.test.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG.test.log; [ $rc -eq 0 ] || exit $rc
i=0
for ENVS in "$@"; do
  i=$((i+1)); [ "$ENVS" = "-" ] && ENVS=""
  echo "== variant $i: $ENVS"
  ( cd /tmp && export TMPDIR=/tmp && env $ENVS timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      -d $R/gpurun_out/${TAG}_v${i}_trace -o run --output-format csv -- \
      python3 $R/bench.py --no-cpu --no-extras --latent 128 --cells 100000 --dtype $DT --steps 20 --warmup 5 --kernel-steps 1 \
      > $R/gpurun_out/${TAG}_v${i}.json 2> $R/gpurun_out/${TAG}_v${i}.err ) || { tail -5 gpurun_out/${TAG}_v${i}.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_v${i}.json'));print(d['value'], d['ms_per_step'], d['kernel_ms'])"
done
