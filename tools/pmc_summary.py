#!/usr/bin/env python3
"""Per-kernel averages of the counters collected by tools/gpu_counters.sh.

    python tools/pmc_summary.py gpurun_out/pmc_<tag>_<cfg> [kernel-substring]
"""
import csv
import glob
import sys
from collections import defaultdict


def load(d, pat):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{d}/*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if pat and pat not in k:
                continue
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def main():
    d = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else None
    for k, cs in load(d, pat).items():
        if "rocclr" in k:
            continue
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        print(k[:90])
        for c in sorted(m):
            print(f"   {c:28s} {m[c]:16.1f}")
        g = lambda c: m.get(c, float("nan"))
        print("   -- derived")
        print(f"   VALU lane util            {g('SQ_THREAD_CYCLES_VALU') / (64 * g('SQ_ACTIVE_INST_VALU')):.3f}")
        print(f"   wait/busy (per wave-cyc)  {g('SQ_WAIT_INST_ANY') / g('SQ_WAVE_CYCLES'):.3f}")
        print(f"   valu/wave-cyc             {g('SQ_ACTIVE_INST_VALU') / g('SQ_WAVE_CYCLES'):.3f}")
        print(f"   avg waves resident/CU-ish {g('SQ_LEVEL_WAVES') / max(g('SQ_BUSY_CYCLES'), 1):.2f}")
        print(f"   vmem in flight per wave   {g('SQ_INST_LEVEL_VMEM') / max(g('SQ_WAVE_CYCLES'), 1):.2f}")
        print(f"   L2 hit                    {g('TCC_HIT_sum') / (g('TCC_HIT_sum') + g('TCC_MISS_sum')):.3f}")
        print(f"   VALU insts per wave       {g('SQ_INSTS_VALU') / g('SQ_WAVES'):.0f}")
        print(f"   VMEM rd per wave          {g('SQ_INSTS_VMEM_RD') / g('SQ_WAVES'):.0f}")
        print(f"   TA busy / GPU busy        {g('TA_BUSY_avr') / g('GRBM_GUI_ACTIVE'):.3f}")
        print(f"   L1 (TCP) hit              {1 - g('TCP_TCC_READ_REQ_sum') / g('TCP_TOTAL_CACHE_ACCESSES_sum'):.3f}")


if __name__ == "__main__":
    main()
