#!/bin/bash
# Round 6: the list-format suite + NB / vMF / tiling / graph / stream parity, then the headline benches
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
TAG=$1
timeout -k 10 600 python -u -m pytest tests/test_gpu_lists.py tests/test_gpu_nb.py tests/test_gpu_tiling.py tests/test_gpu_graph.py tests/test_gpu_vmf.py tests/test_gpu_stream.py tests/test_gpu_dec3.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG.test.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG.test.log; [ $rc -eq 0 ] || exit $rc
for dt in bf16x3 bf16; do
timeout -k 10 200 python bench.py --no-extras --no-cpu --dtype $dt --steps 300 > gpurun_out/$TAG.$dt.json 2>gpurun_out/$TAG.err || { tail -3 gpurun_out/$TAG.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/$TAG.$dt.json'));print('$dt', round(d['value']), d['ms_per_step'], {k: round(v*1e3,1) for k, v in d['kernel_ms'].items()})"
done
timeout -k 10 200 python bench.py --model vmf --no-extras --no-cpu --steps 300 > gpurun_out/$TAG.vmf.json 2>gpurun_out/$TAG.err || { tail -3 gpurun_out/$TAG.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/$TAG.vmf.json'));print('vmf', round(d['value']), d['ms_per_step'], {k: round(v*1e3,1) for k, v in d['kernel_ms'].items()})"
