#!/bin/bash
# rocprofv3 kernel-trace stats of the headline bench alone (no secondary lines), NB and vMF.
# Usage: bash tools/prof_clean.sh TAG [dtype]
TAG=${1:-pc}; DT=${2:-bf16x3}
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd /tmp; export TMPDIR=/tmp
for m in nb vmf; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_${m} -o run --output-format csv -- python3 $R/bench.py --model $m --dtype $DT --no-cpu --no-extras --steps 300 --warmup 20 > $R/gpurun_out/${TAG}_${m}.json 2>$R/gpurun_out/${TAG}_${m}.err || exit 1
done
