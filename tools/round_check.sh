#!/bin/bash
# One GPU call: parity tests -> bench (with CPU baseline) -> rocprofv3 kernel-trace stats.
# Usage: bash tools/round_check.sh TAG
TAG=${1:-run}
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$TAG.test.log 2>&1 || { tail -30 gpurun_out/$TAG.test.log; exit 1; }
tail -3 gpurun_out/$TAG.test.log
timeout -k 10 300 python bench.py > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err || { tail gpurun_out/$TAG.bench.err; exit 2; }
cat gpurun_out/$TAG.bench.json
export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_trace -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 30 --warmup 5 > $R/gpurun_out/${TAG}_trace.json 2>$R/gpurun_out/${TAG}_trace.err || exit 3
find $R/gpurun_out/${TAG}_trace -name "*stats*"
