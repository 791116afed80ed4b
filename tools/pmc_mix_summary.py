"""Per-kernel instruction mix / MFMA utilisation from the rocprofv3 SQ passes of tools/gpu_pmc_mix.sh.

Counters are per dispatch, summed over the chip.  Derived (per dispatch):
  f64_valu_flops = 64 x (2 FMA + MUL + ADD) F64 VALU instructions (all lanes counted as active)
  f64_mfma_flops = 512 x SQ_INSTS_VALU_MFMA_MOPS_F64 (MOPS are units of 512 flops)
  wait_frac      = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (share of wave time waiting on any dependency)
  valu_frac      = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (share of wave time issuing VALU)
usage: python tools/pmc_mix_summary.py gpurun_out/pmcmix out.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    base = name.replace("(anonymous namespace)::", "").split("(")[0]
    return base.replace("void ", "").replace("vio360::", "").strip()


def load(pass_dir):
    vals = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(path, newline="") as f:
            for row in csv.DictReader(f):
                vals[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return vals


def main(src, dst):
    out = {}
    legs = sorted({os.path.basename(d)[:-3] for d in glob.glob(os.path.join(src, "*_p1"))}) or ["mono", "ph", "gba"]
    for leg in legs:
        merged = defaultdict(dict)
        for p in ("p1", "p2"):
            for k, ctrs in load(os.path.join(src, f"{leg}_{p}")).items():
                for c, v in ctrs.items():
                    merged[k][c] = sum(v) / len(v)
                    merged[k]["dispatches"] = len(v)
        for k, c in merged.items():
            g = c.get
            valu = 64.0 * (2 * g("SQ_INSTS_VALU_FMA_F64", 0) + g("SQ_INSTS_VALU_MUL_F64", 0) + g("SQ_INSTS_VALU_ADD_F64", 0))
            mfma = 512.0 * g("SQ_INSTS_VALU_MFMA_MOPS_F64", 0)
            wc = g("SQ_WAVE_CYCLES", 0) or float("nan")
            c.update({"f64_valu_flops": valu, "f64_mfma_flops": mfma,
                      "wait_frac": g("SQ_WAIT_INST_ANY", 0) / wc, "valu_frac": g("SQ_ACTIVE_INST_VALU", 0) / wc,
                      "parked_frac": g("SQ_WAIT_ANY", 0) / wc})
            # MFMA pipe busy over the kernel's GPU-active cycles, per SIMD of the chip (256 CUs x 4):
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs, SQ_VALU_MFMA_BUSY_CYCLES over the 1024 SIMDs
            if g("GRBM_GUI_ACTIVE", 0):
                c["kernel_cycles"] = g("GRBM_GUI_ACTIVE") / 8.0
                c["mfma_busy_frac_chip"] = g("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (c["kernel_cycles"] * 1024.0)
            out[f"{leg}:{k}"] = dict(c)
    with open(dst, "w") as f:
        json.dump({"source": "rocprofv3 --pmc SQ passes (tools/gpu_pmc_mix.sh, tools/gpu_r5_prof.sh)",
                   "commit": os.environ.get("VIO_COMMIT"), "kernels": out}, f, indent=1, sort_keys=True)
    for k, c in sorted(out.items()):
        if c.get("SQ_WAVE_CYCLES", 0) < 1e6:
            continue
        print(f"{k:52s} n={c['dispatches']:4d} valuF64={c['f64_valu_flops'] / 1e9:8.3f}G mfmaF64={c['f64_mfma_flops'] / 1e9:8.3f}G "
              f"VALU_insts={c.get('SQ_INSTS_VALU', 0) / 1e6:9.2f}M VMEM={c.get('SQ_INSTS_VMEM', 0) / 1e6:7.2f}M "
              f"LDS={c.get('SQ_INSTS_LDS', 0) / 1e6:7.2f}M wait={c['wait_frac']:.2f} valu={c['valu_frac']:.2f} "
              f"mfma_busy={c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / 1e6:8.2f}M")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
