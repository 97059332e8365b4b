#!/bin/bash
# Streamed-mode probes: gather-grid sweep (MMVAE_GATHER_WGS) and one kernel trace of the overlap.
# Usage: bash tools/stream_sweep.sh TAG ["wgs list"]
TAG=${1:-ss}; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for g in ${2:-"32 64 128 256"}; do
  MMVAE_GATHER_WGS=$g timeout -k 10 200 python tools/streamed_probe.py > gpurun_out/$TAG.json 2>gpurun_out/$TAG.err || { tail -3 gpurun_out/$TAG.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/$TAG.json'));print('wgs $g', {k: d[k] for k in d if k in ('value','ms_per_step','kernel_ms')})"
done
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/${TAG}_tr -o run --output-format csv -- python3 $R/tools/streamed_probe.py > /dev/null 2>>$R/gpurun_out/$TAG.err || exit 2
f=$(python3 -c "import glob,sys; print(glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0])" $R/gpurun_out/${TAG}_tr)
python3 $R/tools/trace_overlap.py $f
python3 - $f <<'PY'
import csv, sys, collections
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
st = collections.defaultdict(list)
for r in rows: st[r["Kernel_Name"][:28]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(st.items(), key=lambda kv: -sum(kv[1])):
    if len(v) > 5: print("%-28s n=%4d avg %.1f us (last 20 avg %.1f)" % (k, len(v), sum(v)/len(v), sum(v[-20:])/len(v[-20:])))
# one step's timeline near the end
tl = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:22]) for r in rows[-40:]]
t0 = tl[0][0]
for s, e, n in tl: print("%9.1f %9.1f %s" % ((s - t0) / 1e3, (e - t0) / 1e3, n))
PY
rm -rf $R/gpurun_out/${TAG}_tr
