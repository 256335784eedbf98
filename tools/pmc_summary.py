"""Summarise tools/gpu_pmc3.sh output: render-kernel counters and derived ratios.

python tools/pmc_summary.py gpurun_out/pmc [stats.json]
"""
import csv
import glob
import json
import os
import sys


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    c = {}
    for f in glob.glob(os.path.join(d, "p*", "*_counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            if "render_kernel" not in row["Kernel_Name"]:
                continue
            c[row["Counter_Name"]] = c.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    for k in sorted(c):
        print(f"{k:28s} {c[k]:.4e}")
    g = c.get
    if g("SQ_ACTIVE_INST_VALU") and g("SQ_THREAD_CYCLES_VALU"):
        print(f"VALU lane utilisation        {g('SQ_THREAD_CYCLES_VALU') / (64 * g('SQ_ACTIVE_INST_VALU')):.3f}")
    if g("SQ_WAVES") and g("SQ_INSTS_VALU"):
        print(f"VALU instr per wave          {g('SQ_INSTS_VALU') / g('SQ_WAVES'):.4e}")
    if g("SQ_WAIT_INST_ANY") and g("SQ_WAVE_CYCLES"):
        print(f"wait_inst_any / wave_cycles  {g('SQ_WAIT_INST_ANY') / g('SQ_WAVE_CYCLES'):.3f}")
    if g("SQ_WAIT_ANY") and g("SQ_WAVE_CYCLES"):
        print(f"wait_any / wave_cycles       {g('SQ_WAIT_ANY') / g('SQ_WAVE_CYCLES'):.3f}")
    if g("FETCH_SIZE"):
        print(f"FETCH bytes (x1024, x2 gfx950 correction) {g('FETCH_SIZE') * 1024 * 2:.4e}")
    if g("WRITE_SIZE"):
        print(f"WRITE bytes (x1024)          {g('WRITE_SIZE') * 1024:.4e}")


if __name__ == "__main__":
    main()
