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
    # per pass, the counter's sum over the render-kernel dispatches; a counter collected in several
    # passes (SQ_WAVE_CYCLES, SQ_INSTS_VMEM_RD) is the mean of its passes, not their sum
    passes = {}
    for f in glob.glob(os.path.join(d, "p*", "*_counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            if "render_kernel" not in row["Kernel_Name"]:
                continue
            pc = passes.setdefault(row["Counter_Name"], {})
            pc[f] = pc.get(f, 0.0) + float(row["Counter_Value"])
    c = {k: sum(v.values()) / len(v) for k, v in passes.items()}
    for k in sorted(c):
        print(f"{k:28s} {c[k]:.4e}")
    g = c.get
    if g("SQ_ACTIVE_INST_VALU") and g("SQ_THREAD_CYCLES_VALU"):
        print(f"VALU lane utilisation        {g('SQ_THREAD_CYCLES_VALU') / (64 * g('SQ_ACTIVE_INST_VALU')):.3f}")
    if g("SQ_LDS_BANK_CONFLICT") is not None and g("SQ_LDS_IDX_ACTIVE"):
        print(f"LDS bank conflict / LDS-active cycles {g('SQ_LDS_BANK_CONFLICT') / g('SQ_LDS_IDX_ACTIVE'):.3f}")
    if g("SQ_WAVES") and g("SQ_INSTS_VALU"):
        print(f"VALU instr per wave          {g('SQ_INSTS_VALU') / g('SQ_WAVES'):.4e}")
    if g("SQ_WAIT_INST_ANY") and g("SQ_WAVE_CYCLES"):
        print(f"wait_inst_any / wave_cycles  {g('SQ_WAIT_INST_ANY') / g('SQ_WAVE_CYCLES'):.3f}")
    if g("SQ_WAIT_ANY") and g("SQ_WAVE_CYCLES"):
        print(f"wait_any / wave_cycles       {g('SQ_WAIT_ANY') / g('SQ_WAVE_CYCLES'):.3f}")
    if g("TCP_TCC_READ_REQ_sum") and g("TCP_TCC_READ_REQ_LATENCY_sum"):
        print(f"L1->L2 read latency (cycles) {g('TCP_TCC_READ_REQ_LATENCY_sum') / g('TCP_TCC_READ_REQ_sum'):.1f}")
    if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum"):
        print(f"L2 hit rate                  {g('TCC_HIT_sum') / (g('TCC_HIT_sum') + g('TCC_MISS_sum')):.3f}")
    if g("SQ_INST_LEVEL_VMEM") and g("SQ_INSTS_VMEM_RD"):
        print(f"VMEM level / VMEM reads      {g('SQ_INST_LEVEL_VMEM') / g('SQ_INSTS_VMEM_RD'):.1f}  (mean cycles a read is in flight x4)")
    if g("SQ_INSTS_VMEM_RD") and g("SQ_INSTS_VALU"):
        print(f"VMEM reads / VALU            {g('SQ_INSTS_VMEM_RD') / g('SQ_INSTS_VALU'):.4f}")
    if g("FETCH_SIZE"):
        print(f"FETCH bytes (x1024, x2 gfx950 correction) {g('FETCH_SIZE') * 1024 * 2:.4e}")
    if g("WRITE_SIZE"):
        print(f"WRITE bytes (x1024)          {g('WRITE_SIZE') * 1024:.4e}")


if __name__ == "__main__":
    main()
