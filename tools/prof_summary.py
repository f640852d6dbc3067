"""Markdown table of a rocprofv3 --stats kernel summary (for profiles/).

usage: python tools/prof_summary.py <run_kernel_stats.csv> <out.md> "<title>" "<command>" [top]
Copies the csv next to the markdown (<out>_kernel_stats.csv).
"""
import csv
import shutil
import sys


def main():
    src, out, title, cmd = sys.argv[1:5]
    top = int(sys.argv[5]) if len(sys.argv) > 5 else 15
    rows = list(csv.DictReader(open(src)))
    lines = [f"# {title}", "", f"Command: `{cmd}`", "",
             "| kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|"]
    for r in rows[:top]:
        name = r["Name"].replace("|", "/")
        lines.append(f"| `{name[:90]}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
                     f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.1f} |")
    open(out, "w").write("\n".join(lines) + "\n")
    shutil.copy(src, out[:-3] + "_kernel_stats.csv" if out.endswith(".md") else out + "_kernel_stats.csv")


if __name__ == "__main__":
    main()
