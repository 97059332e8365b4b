"""Per-dispatch durations of the last full step in a rocprofv3 kernel trace (between the last two
k_adam dispatches).   Usage: python tools/trace_step.py TRACE_CSV [min_us]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
mn = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
idx = [i for i, r in enumerate(rows) if "k_adam" in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
tot = 0.0
for r in rows[a + 1:b + 1]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    tot += d
    if d >= mn:
        g = (int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), r["Grid_Size_Y"], r["Grid_Size_Z"])
        print(f"{d:8.1f} grid={g} vgpr={r['VGPR_Count']}/{r['Accum_VGPR_Count']} scr={r['Scratch_Size']} "
              f"{r['Kernel_Name'][:80]}")
print(f"sum {tot:.1f} us")
