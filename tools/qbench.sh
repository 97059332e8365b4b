# quick headline numbers (no profiler): value / ms per step / device ms per step per dtype
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for dt in ${DTYPES:-bf16x3 bf16}; do
  timeout -k 10 300 python bench.py --no-extras --no-cpu --dtype $dt --steps ${STEPS:-200} ${BENCH_ARGS:-} > gpurun_out/q_$dt.json 2>gpurun_out/q_$dt.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/q_$dt.json'));print('$dt', round(d['value']), d['ms_per_step'], d['device_ms_per_step'], d.get('median_ms_per_step_synced'))"
done
