"""Summarise tools/pmc.sh output: per kernel mean duration and counters per dispatch.

    python tools/pmc_summary.py ROOT TAG [KEY_PREFIX]
With KEY_PREFIX (e.g. nb/bf16) the per-launch HBM traffic of every kernel is also written to
ROOT/TAG_traffic.json as {"KEY_PREFIX/kernel": bytes} (FETCH_SIZE doubled: gfx950 counts 64 B
per 128-B streaming request, MI355X_MICROARCH.md §HBM; both counters are KiB)."""
import collections, csv, glob, json, os, sys

root, tag = sys.argv[1], sys.argv[2]
prefix = sys.argv[3] if len(sys.argv) > 3 else None
traffic = {}


def short(n):
    import re
    m = re.match(r"_ZN5mmvae(\d+)", n)
    if m:  # mangled template instance: keep the kernel's own name
        L = int(m.group(1))
        return n[m.end():m.end() + L]
    n = n.split("(")[0].replace("void ", "")
    for a, b in (("mmvae::", ""), ("__bf16", "bf16")):
        n = n.replace(a, b)
    return n[:40]


dur = collections.defaultdict(list)
for f in glob.glob(os.path.join(root, f"{tag}_trace", "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
cnt = collections.defaultdict(lambda: collections.defaultdict(list))
for p in ("p1", "p2", "p3", "p4"):
    for f in glob.glob(os.path.join(root, f"{tag}_{p}", "**", "*counter_collection.csv"), recursive=True):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            per[(short(r["Kernel_Name"]), r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (k, _, c), v in per.items():
            cnt[k][c].append(v)
ks = sorted(dur, key=lambda k: -sum(dur[k]) / len(dur[k]))
for k in ks:
    d = sum(dur[k]) / len(dur[k])
    c = {n: sum(v) / len(v) for n, v in cnt[k].items()}
    line = f"{k:40s} {d:8.1f} us  n={len(dur[k]):4d}"
    if c:
        waves = max(c.get("SQ_WAVES", 1), 1)
        if "SQ_INSTS_VALU" in c:
            line += f" | VALU/wave {c['SQ_INSTS_VALU'] / waves:8.0f} SALU/wave {c.get('SQ_INSTS_SALU', 0) / waves:6.0f}"
        if "SQ_WAVE_CYCLES" in c:
            wc = c["SQ_WAVE_CYCLES"]
            line += f" wait {c.get('SQ_WAIT_ANY', 0) / wc:4.2f} waitinst {c.get('SQ_WAIT_INST_ANY', 0) / wc:4.2f} valu-act {c.get('SQ_ACTIVE_INST_VALU', 0) / wc:4.2f}"
        if "SQ_INSTS_LDS" in c:
            line += f" | LDS/wave {c['SQ_INSTS_LDS'] / waves:6.0f} bankconf/idx {c.get('SQ_LDS_BANK_CONFLICT', 0) / max(c.get('SQ_LDS_IDX_ACTIVE', 1), 1):4.2f} trans/wave {c.get('SQ_INSTS_VALU_TRANS_F32', 0) / waves:6.0f} mfma/wave {c.get('SQ_INSTS_MFMA', 0) / waves:5.0f}"
        if "FETCH_SIZE" in c:
            # gfx950: FETCH_SIZE counts 64 B per 128-B request (MI355X_MICROARCH.md) -> x2, KB -> MB
            line += f" | fetch {2 * c['FETCH_SIZE'] / 1024:7.1f} MB write {c.get('WRITE_SIZE', 0) / 1024:6.1f} MB"
            if prefix:  # instances sharing a name (e.g. pass B's loss-only one): the longest-running
                traffic.setdefault(f"{prefix}/{k.split('<')[0]}", (2 * c["FETCH_SIZE"] + c.get("WRITE_SIZE", 0)) * 1024.0)
    print(line)
if prefix:
    json.dump(traffic, open(os.path.join(root, f"{tag}_traffic.json"), "w"), indent=1, sort_keys=True)
