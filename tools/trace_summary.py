"""Per-step kernel time by (kernel, grid) from a rocprofv3 kernel_trace.csv.
    python tools/trace_summary.py gpurun_out/TAG_trace/run_kernel_trace.csv KERNEL_PER_STEP [top]
KERNEL_PER_STEP: a kernel name launched exactly once per step (normalises the totals)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
per = sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
agg = collections.defaultdict(lambda: [0, 0.0])
nstep = 0
for r in rows:
    n = r["Kernel_Name"]
    if per in n:
        nstep += 1
    g = (r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    k = (n.split("(")[0][:60], g)
    agg[k][0] += 1
    agg[k][1] += d
tot = sum(v[1] for v in agg.values())
print(f"steps {nstep}, total {tot / nstep:.1f} us/step")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{v[1] / nstep:9.1f} us/step  {v[0] / nstep:5.2f}/step  {v[1] / v[0]:8.1f} us/call  {k[0]} {k[1]}")
