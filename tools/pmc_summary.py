"""Per-launch HBM bytes of each kernel from tools/pmc.sh's counter CSVs.

FETCH_SIZE / WRITE_SIZE are reported by rocprofv3 in KiB per dispatch.  On
gfx950 FETCH_SIZE counts 64 B per 128-B memory request, i.e. half of the bytes
of wide streaming reads: corrected read bytes = 2 x FETCH_SIZE x 1024
(MI355X_MICROARCH.md, HBM [CDNA4]).  WRITE_SIZE is taken as is.
Writes <dir>/pmc_summary.json: {kernel: {launches, read_bytes, write_bytes}}.
"""
import collections
import csv
import glob
import json
import os
import sys


def load(d, counter):
    out = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, counter, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            out[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return out


def main(d):
    fe, wr = load(d, "FETCH_SIZE"), load(d, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fe) | set(wr)):
        f, w = fe.get(k, []), wr.get(k, [])
        res[k] = {"launches": max(len(f), len(w)),
                  "fetch_size_kib_mean": sum(f) / len(f) if f else None,
                  "read_bytes": 2 * 1024 * sum(f) / len(f) if f else None,
                  "write_bytes": 1024 * sum(w) / len(w) if w else None}
    json.dump(res, open(os.path.join(d, "pmc_summary.json"), "w"), indent=1)
    for k, v in sorted(res.items(), key=lambda kv: -(kv[1]["read_bytes"] or 0))[:12]:
        print(f"{v['launches']:5d} {((v['read_bytes'] or 0) / 1e9):8.3f} GB rd {((v['write_bytes'] or 0) / 1e9):8.3f} GB wr  {k[:90]}")


if __name__ == "__main__":
    main(sys.argv[1])
