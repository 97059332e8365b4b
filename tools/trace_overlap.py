"""Overlap of k_stream_gather with the other kernels in a rocprofv3 kernel trace (queue ids and
timestamps).  Usage: python tools/trace_overlap.py gpurun_out/DIR/run_kernel_trace.csv"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40], r.get("Queue_Id", "?"), r.get("Stream_Id", "?")) for r in rows]
ks.sort()
g = [k for k in ks if "stream_gather" in k[2]]
other = [k for k in ks if "stream_gather" not in k[2] and "synth" not in k[2]]
print("gathers", len(g), "queues", sorted(set((k[3], k[4]) for k in g)), "others' queues", sorted(set((k[3], k[4]) for k in other))[:6])
ov = 0
for s, e, *_ in g[-10:]:
    busy = sum(max(0, min(e, e2) - max(s, s2)) for s2, e2, *_ in other)
    ov += busy
    print("gather %.1f us, overlapped by other kernels %.1f us" % ((e - s) / 1e3, busy / 1e3))
