#!/bin/bash
# One GPU call: NB + vMF parity tests, then the NB (and optionally vMF) bench without the CPU leg.
# Usage: bash tools/quick_nb.sh TAG [vmf]
TAG=${1:-q}
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG.test.log 2>&1 || { tail -40 gpurun_out/$TAG.test.log; exit 1; }
tail -2 gpurun_out/$TAG.test.log
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err || { tail gpurun_out/$TAG.bench.err; exit 2; }
cat gpurun_out/$TAG.bench.json
if [ "$2" == "vmf" ]; then
  timeout -k 10 300 python bench.py --no-cpu --model vmf > gpurun_out/$TAG.bench_vmf.json 2> gpurun_out/$TAG.bench_vmf.err || { tail gpurun_out/$TAG.bench_vmf.err; exit 3; }
  cat gpurun_out/$TAG.bench_vmf.json
fi
