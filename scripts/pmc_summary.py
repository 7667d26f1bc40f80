#!/usr/bin/env python
"""Summarise a rocprofv3 --pmc counter_collection.csv into a markdown table: per kernel,
the mean of each counter over its dispatches plus derived ratios (per-wave instruction
counts, MFMA busy share, LDS bank conflicts per LDS instruction)."""
import csv
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"srnn::(k_\w+)<srnn::(\w+)<([\d, ]+)>(?:, (\d+))?", name)
    if m:
        return f"{m.group(1)}<{m.group(2)}<{m.group(3)}>{', ' + m.group(4) if m.group(4) else ''}>"
    return name[:60]


def main(path, title="", only=None):
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in csv.DictReader(open(path)):
        if only and only not in r["Kernel_Name"]:
            continue
        k = short(r["Kernel_Name"])
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    print(f"### {title}\n")
    counters = sorted({c for v in per.values() for c in v})
    print("| kernel | dispatches | " + " | ".join(counters) + " | derived |")
    print("|---|---:|" + "---:|" * len(counters) + "---|")
    for k, v in sorted(per.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CYCLES", kv[1].get("SQ_WAVES", 0))):
        n = len(disp[k])
        der = []
        waves = v.get("SQ_WAVES", 0)
        if waves:
            if "SQ_INSTS_VALU" in v:
                der.append(f"VALU/wave {v['SQ_INSTS_VALU'] / waves:.0f}")
            if "SQ_INSTS_MFMA" in v:
                der.append(f"MFMA/wave {v['SQ_INSTS_MFMA'] / waves:.0f}")
            if "SQ_INSTS_LDS" in v:
                der.append(f"LDS/wave {v['SQ_INSTS_LDS'] / waves:.0f}")
        if v.get("SQ_VALU_MFMA_BUSY_CYCLES") and v.get("GRBM_GUI_ACTIVE"):
            # MFMA-busy cycles (sum over SIMDs of the issued MFMAs' cycles) vs. SIMD-cycles
            # of the dispatch: GRBM_GUI_ACTIVE is summed over the 8 XCDs; 1024 SIMDs
            der.append(f"MFMA busy {v['SQ_VALU_MFMA_BUSY_CYCLES'] / (v['GRBM_GUI_ACTIVE'] / 8 * 1024):.1%}")
        if v.get("SQ_LDS_BANK_CONFLICT") is not None and v.get("SQ_INSTS_LDS"):
            der.append(f"bank-conflict cyc/LDS instr {v['SQ_LDS_BANK_CONFLICT'] / v['SQ_INSTS_LDS']:.2f}")
        if v.get("SQ_ACTIVE_INST_VALU") and v.get("SQ_WAIT_ANY") is not None:
            der.append(f"wait/valu-active {v['SQ_WAIT_ANY'] / max(v['SQ_ACTIVE_INST_VALU'], 1):.2f}")
        print(f"| `{k}` | {n} | " + " | ".join(f"{v.get(c, 0) / n:.3g}" for c in counters) + " | " +
              "; ".join(der) + " |")
    print()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else sys.argv[1], sys.argv[3] if len(sys.argv) > 3 else None)
