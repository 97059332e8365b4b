#!/bin/bash
# One GPU call: parity tests -> NB and vMF benches (with CPU baseline) -> rocprofv3 kernel-trace
# stats of the default bench.   Usage: bash tools/round_check.sh TAG [skip-tests]
TAG=${1:-run}
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$TAG.test.log 2>&1 || { tail -30 gpurun_out/$TAG.test.log; exit 1; }
  tail -2 gpurun_out/$TAG.test.log
fi
timeout -k 10 300 python bench.py > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err || { tail gpurun_out/$TAG.bench.err; exit 2; }
cat gpurun_out/$TAG.bench.json
timeout -k 10 300 python bench.py --model vmf > gpurun_out/$TAG.bench_vmf.json 2> gpurun_out/$TAG.bench_vmf.err || { tail gpurun_out/$TAG.bench_vmf.err; exit 3; }
cat gpurun_out/$TAG.bench_vmf.json
export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_trace -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 30 --warmup 5 > $R/gpurun_out/${TAG}_trace.json 2>$R/gpurun_out/${TAG}_trace.err || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_vtrace -o run --output-format csv -- python3 $R/bench.py --model vmf --no-cpu --steps 30 --warmup 5 > $R/gpurun_out/${TAG}_vtrace.json 2>$R/gpurun_out/${TAG}_vtrace.err || exit 5
# keep the merged-back output small (gpurun copies at most 64 MiB): the per-dispatch traces go
rm -f $R/gpurun_out/${TAG}_trace/run_kernel_trace.csv $R/gpurun_out/${TAG}_vtrace/run_kernel_trace.csv
