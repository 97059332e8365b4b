# Round-2 closing run: GPU suite + smoke, the default bench (headline + extras + CPU baseline),
# rocprofv3 kernel-trace stats of the same command (x3 headline) and of the vMF bench.
TAG=${1:-r2_s3}
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG.test.log 2>&1 || { tail -30 gpurun_out/$TAG.test.log; exit 1; }
tail -2 gpurun_out/$TAG.test.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 2
timeout -k 10 400 python bench.py > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err || { tail gpurun_out/$TAG.bench.err; exit 3; }
python -c "import json;d=json.load(open('gpurun_out/$TAG.bench.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['full_loop']['value'])"
export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_trace -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-extras --steps 30 --warmup 5 > $R/gpurun_out/${TAG}_trace.json 2>$R/gpurun_out/${TAG}_trace.err || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_vtrace -o run --output-format csv -- python3 $R/bench.py --model vmf --cells 100000 --no-cpu --no-extras --steps 30 --warmup 5 > $R/gpurun_out/${TAG}_vtrace.json 2>$R/gpurun_out/${TAG}_vtrace.err || exit 5
echo done
