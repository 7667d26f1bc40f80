#!/usr/bin/env python
"""Markdown summary of a scripts/gpu_r4.sh run (gpurun_out/*_<tag>.log + the rocprofv3 stats CSV).

usage: python scripts/r4_report.py <tag> > profiles/r4x_<name>.md
"""
import csv
import glob
import json
import os
import re
import sys

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")


def jlines(path):
    out = []
    if not os.path.exists(path):
        return out
    for line in open(path):
        line = line.strip()
        if line.startswith("{"):
            try:
                out.append(json.loads(line))
            except json.JSONDecodeError:
                pass
    return out


def short(name):
    name = re.sub(r"srnn::", "", name)
    name = re.sub(r"\(SrnnCfg, SrnnArgs.*", "", name)
    name = re.sub(r"void ", "", name)
    return name[:90]


def main(tag):
    print(f"# GPU run `{tag}` (scripts/gpu_r4.sh, one MI355X)\n")
    p = os.path.join(OUT, f"pytest_{tag}.log")
    if os.path.exists(p):
        last = [l for l in open(p) if re.search(r"\d+ passed|failed", l)]
        print("## Tests\n\n`" + (last[-1].strip() if last else "?") + "`\n")
    b = jlines(os.path.join(OUT, f"bench_{tag}.log"))
    if b:
        d = b[-1]
        c = d["config"]
        print("## Headline (bench.py --steps 20 --warmup 5)\n")
        print(f"* synchronous order: **{d['ms_per_step']:.4f} ms / generation**, {d['value']:.3e} "
              f"particle-generations/s, census {c['final_census']}")
        ro = c.get("reference_order")
        if ro:
            print(f"* reference (sequential) order, same soup: **{ro['ms_per_step']:.4f} ms / generation**, "
                  f"{ro['value']:.3e} particle-generations/s, levels {ro['levels']}")
        print(f"* execution: `{json.dumps(c.get('execution'))}`\n")
    rows = []
    for f in sorted(glob.glob(os.path.join(OUT, f"strong_*_{tag}.log"))):
        m = re.search(r"strong_(\d+)_(\d+)_", os.path.basename(f))
        js = jlines(f)
        if m and js:
            rows.append((int(m.group(1)), int(m.group(2)), js[-1]["ms_per_step"], js[-1]["config"]["global_batch"]))
    if rows:
        print("## Strong-scaling model: one rank of an N-rank 100k soup (forced-sharded, remote fraction emulated)\n")
        print("| N | slots per rank | lanes per particle | ms / generation (rank) |\n|---:|---:|---:|---:|")
        for r in sorted(rows):
            print(f"| {r[0]} | {r[3]} | {r[1]} | {r[2]:.4f} |")
        print()
    s = jlines(os.path.join(OUT, f"pairs_{tag}.log"))
    if s:
        print("## Lanes per particle vs population size (ms / generation, 20-generation graphs)\n")
        print("| order | n | 1 lane | 2 lanes | pair speedup |\n|---|---:|---:|---:|---:|")
        by = {}
        for r in s:
            by.setdefault((r["order"], r["n"]), {})[r["lanes"]] = r["ms_per_gen"]
        for (o, n), v in sorted(by.items()):
            if 1 in v and 2 in v:
                print(f"| {o} | {n} | {v[1]:.4f} | {v[2]:.4f} | {v[1] / v[2]:.2f}x |")
        print()
    for kind in ("reg", "lds"):
        sh = jlines(os.path.join(OUT, f"shapes_{kind}_{tag}.log"))
        if sh:
            print(f"## Shapes ({'register' if kind == 'reg' else 'LDS'} SGD of the wide Weightwise wave kernels)\n")
            for r in sh:
                print("* `" + json.dumps(r) + "`")
            print()
    for f in glob.glob(os.path.join(OUT, f"prof_{tag}", "**", "*kernel_stats.csv"), recursive=True):
        rr = list(csv.DictReader(open(f)))
        tot = sum(float(r["TotalDurationNs"]) for r in rr)
        print(f"## Kernel trace ({os.path.relpath(f, OUT)})\n")
        print("| kernel | calls | total us | avg us | % |\n|---|---:|---:|---:|---:|")
        for r in sorted(rr, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
            t = float(r["TotalDurationNs"])
            print(f"| `{short(r['Name'])}` | {r['Calls']} | {t / 1e3:.1f} | {float(r['AverageNs']) / 1e3:.2f} | "
                  f"{100 * t / max(tot, 1):.1f} |")
        print()


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r4")
