#!/bin/bash
# Closing evidence of a build in one GPU call: the full GPU suite, the default NB bench (every line,
# CPU baseline), the vMF bench, the driver's 20/5 command, rocprofv3 kernel stats of the NB and
# vMF x3 headline benches, and PMC passes (tools/pmc.sh) of both.
# Usage: bash tools/closing.sh TAG [skip-tests]
TAG=${1:-close}
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1
  rc=$?; tail -2 gpurun_out/${TAG}_gpu_tests.txt; [ $rc -eq 0 ] || exit 1
fi
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench_nb.json 2> gpurun_out/${TAG}_bench_nb.err || { tail gpurun_out/${TAG}_bench_nb.err; exit 2; }
timeout -k 10 300 python bench.py --model vmf > gpurun_out/${TAG}_bench_vmf.json 2> gpurun_out/${TAG}_bench_vmf.err || { tail gpurun_out/${TAG}_bench_vmf.err; exit 3; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_nb_short_window.json 2> gpurun_out/${TAG}_short.err || exit 4
bash tools/prof_clean.sh ${TAG}_prof bf16x3 || exit 5
bash tools/pmc.sh ${TAG}_pmc_nb nb bf16x3 > /dev/null || exit 6
bash tools/pmc.sh ${TAG}_pmc_vmf vmf bf16x3 > /dev/null || exit 7
rm -f gpurun_out/${TAG}_prof_*/run_kernel_trace.csv
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_nb.json'));print(d['value'], d['ms_per_step'], d['roofline']);d=json.load(open('gpurun_out/${TAG}_bench_vmf.json'));print('vmf', d['value'], d['ms_per_step']);d=json.load(open('gpurun_out/${TAG}_bench_nb_short_window.json'));print('short', d['value'], d['ms_per_step'])"
