"""Markdown table of tools/robustness.py results (JSON lines).

usage: python tools/robustness_table.py results.jsonl [more.jsonl ...]
Later lines for the same (problem, N, pc type, option set) replace earlier ones.
"""
import json
import sys

REASON = {2: "rtol", 3: "atol", -3: "max its", -100: "time limit", -4: "dtol", -5: "breakdown", -8: "indefinite PC",
          -9: "nan/inf", -11: "PC failed"}


def main(paths):
    rows = {}
    for p in paths:
        for line in open(p):
            line = line.strip()
            if not line.startswith("{"):
                continue
            d = json.loads(line)
            rows[(d["problem"], d["options"], d["pc_type"], d["N"])] = d
    print("| problem | options | pc type | N | DoF | its | reason | rnorm / rnorm0 | setup s | solve s | inner solves: its (mean / max) |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    for k in sorted(rows, key=lambda k: (k[0], k[1], k[2], k[3])):
        d = rows[k]
        inner = []
        for pre, v in d["inner"].items():
            if v["its"] > v["solves"]:  # skip PREONLY (one "iteration" per solve)
                last = REASON.get(v.get("last_negative"), v.get("last_negative"))
                neg = f", {v['negative_reason']} diverged" + (f": {last}" if v.get("last_negative") else "") \
                    if v["negative_reason"] else ""
                inner.append(f"{pre.rstrip('_')} {v['its']} ({v['its'] / v['solves']:.0f} / {v['max']}{neg})")
        red = (d["rnorm"] / d["rnorm0"]) if d.get("rnorm0") else float("nan")
        print(f"| {d['problem']} | {d['options']} | {d['pc_type']} | {d['N']} | {d['dofs']:,} | {d['its']} | "
              f"{REASON.get(d['reason'], d['reason'])} | {red:.1e} | {d['setup_s']} | {d['solve_s']} | "
              f"{'; '.join(inner) or '-'} |")


if __name__ == "__main__":
    main(sys.argv[1:])
