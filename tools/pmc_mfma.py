"""Summarise a rocprofv3 --pmc pass of MFMA counters per (kernel, grid):
python tools/pmc_mfma.py <run_counter_collection.csv> [name-filter ...]

Counters (one pass: SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16
SQ_INSTS_VALU_MFMA_BF16 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE).  Per dispatch:
  flop      = SQ_INSTS_VALU_MFMA_MOPS_BF16 * 512 (MOPS unit; cross-checked below
              against 16384 FLOP per v_mfma_f32_16x16x32_bf16 instruction)
  tflops    = flop / dispatch duration
  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs): the
              fraction of SIMD-cycles the matrix cores were busy.  GRBM_GUI_ACTIVE
              reads as the sum over the 8 XCDs (with /8 the busy fraction equals
              the MOPS-derived fraction of peak on every MFMA-bound kernel)
  of_peak   = tflops / 2500 (MI355X dense bf16)"""
import collections
import csv
import sys

PEAK = 2500.0


def main():
    path, filt = sys.argv[1], sys.argv[2:]
    per = collections.defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0]
        if filt and not any(f in name for f in filt):
            continue
        d = r["Dispatch_Id"]
        per[d][r["Counter_Name"]] = float(r["Counter_Value"])
        meta[d] = (name, int(r["Grid_Size"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for d, c in per.items():
        name, grid, dt = meta[d]
        a = agg[(name, grid)]
        a["n"] += 1
        a["dt"] += dt
        for k, v in c.items():
            a[k] += v
    print("kernel | grid | launches | avg us | MFMA inst | FLOP/inst | TFLOP/s | of 2.5 PF | MFMA busy")
    for (name, grid), a in sorted(agg.items(), key=lambda x: -x[1]["dt"]):
        inst = a.get("SQ_INSTS_VALU_MFMA_BF16", 0.0)
        mops = a.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0)
        if inst == 0:
            continue
        flop = mops * 512
        tf = flop / a["dt"] / 1e12
        busy = a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / max(a.get("GRBM_GUI_ACTIVE", 1.0) / 8 * 1024, 1.0)
        print(f"{name} | {grid} | {int(a['n'])} | {a['dt'] / a['n'] * 1e6:.1f} | {inst / a['n']:.3g} | "
              f"{flop / inst:.0f} | {tf:.0f} | {tf / PEAK:.3f} | {busy:.3f}")


if __name__ == "__main__":
    main()
