# kernel-trace stats of the headline step (bf16 and x3) + latent-kernel phase stamps
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; export TMPDIR=/tmp; cd /tmp
TAG=${TAG:-r2}
for DT in ${DTYPES:-bf16 bf16x3}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG_$DT -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu --no-extras --dtype $DT ${BENCH_ARGS:-} > $R/gpurun_out/${TAG}_bench_$DT.json 2>$R/gpurun_out/${TAG}_$DT.err || exit 1
  f=$(find $R/gpurun_out/prof_$TAG_$DT -name "*kernel_stats.csv" | head -1); cp $f $R/gpurun_out/${TAG}_${DT}_kernel_stats.csv
  python3 - $R/gpurun_out/${TAG}_${DT}_kernel_stats.csv <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:16]:
    print("%-40s n=%5s avg %8.1f us" % (r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e3))
PY
done
if [ -n "$LAT" ]; then
  cd $R && KER=fwd timeout -k 10 120 python3 tools/stamps_lat.py && KER=bwd timeout -k 10 120 python3 tools/stamps_lat.py
fi
