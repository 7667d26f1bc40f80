#!/usr/bin/env python
"""Summarise a rocprofv3 --kernel-trace --stats CSV into a markdown table (profiles/)."""
import csv
import re
import sys

OPS = {0: "init", 1: "apply", 2: "run_fixpoint", 3: "train", 4: "learn", 5: "classify", 6: "perturb",
       7: "soup_decide", 8: "soup_fill", 9: "soup_evolve", 10: "scan", 11: "respawn", 12: "vary_run"}


def short(name: str) -> str:
    m = re.search(r"srnn::k_op<srnn::(\w+)<([\d, ]+)>, (\d+)>", name)
    if m:
        return f"k_op<{m.group(1)}<{m.group(2)}>, {OPS.get(int(m.group(3)), m.group(3))}>"
    m = re.search(r"srnn::k_classify_count<srnn::(\w+)<([\d, ]+)>", name)
    if m:
        return f"k_classify_count<{m.group(1)}<{m.group(2)}>>"
    if "rocprim" in name:
        return "rocprim scan (" + ("init_lookback" if "init_lookback" in name else "scan") + ")"
    m = re.search(r"at::native::(\w+)<.*?at::native::(\w+)", name)
    if m:
        return f"torch {m.group(1)}<{m.group(2)}>"
    return name[:80]


def main(path, title=""):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"### {title}\n")
    print("| kernel | calls | total us | avg us | % |")
    print("|---|---:|---:|---:|---:|")
    for r in rows:
        print(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['TotalDurationNs'])/1e3:.1f} | "
              f"{float(r['AverageNs'])/1e3:.2f} | {float(r['Percentage']):.1f} |")
    print(f"\ntotal GPU kernel time: {tot/1e3:.1f} us\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else sys.argv[1])
