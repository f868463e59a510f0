"""Executed FP64 work per dispatch of one kernel from a tools/pmc_summary.py text summary.

    python3 tools/pmc_exec.py <pmc_summary.txt> <kernel-substring> [--units-per-dispatch U] [--unit NAME]

Executed flops = SQ_INSTS_VALU_FMA_F64 x 128 + (SQ_INSTS_VALU_ADD_F64 + SQ_INSTS_VALU_MUL_F64) x 64
+ SQ_INSTS_VALU_MFMA_MOPS_F64 x 512 (wave instructions x 64 lanes x 2 / 1 flops; one
v_mfma_f64_16x16x4 = 2048 flops = 4 MOPS).  An upper bound for the VALU part (partially active waves
count as full).  With --units-per-dispatch the JSON also carries executed flops per unit (e.g. per
two-site update), which bench.py multiplies by its live units per launch.
"""
import json
import sys


def parse(path):
    out, cur = {}, None
    with open(path) as fh:
        for line in fh:
            if line.startswith("== "):
                cur = line[3:].strip()
                out[cur] = {}
            elif cur is not None and line.strip():
                parts = line.split()
                if parts[0].startswith("dispatches="):
                    out[cur]["dispatches"] = float(parts[0].split("=")[1])
                    out[cur]["mean_dur_us"] = float(parts[1].split("=")[1])
                else:
                    out[cur][parts[0]] = float(parts[1])
    return out


def main(argv):
    path, ker = argv[0], argv[1]
    units = None
    unit = "update"
    if "--units-per-dispatch" in argv:
        units = float(argv[argv.index("--units-per-dispatch") + 1])
    if "--unit" in argv:
        unit = argv[argv.index("--unit") + 1]
    summ = parse(path)
    name = next(k for k in summ if ker in k)
    c = summ[name]
    fma, add, mul = c.get("SQ_INSTS_VALU_FMA_F64", 0.0), c.get("SQ_INSTS_VALU_ADD_F64", 0.0), c.get("SQ_INSTS_VALU_MUL_F64", 0.0)
    mops = c.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0)
    valu = 128.0 * fma + 64.0 * (add + mul)
    mfma = 512.0 * mops
    ex = valu + mfma
    dur = c["mean_dur_us"] * 1e-6
    rec = {"kernel": ker, "source": path, "mean_dur_us": c["mean_dur_us"],
           "executed_flops_per_dispatch": ex, "valu_flops_per_dispatch": valu, "mfma_flops_per_dispatch": mfma,
           "executed_tflops": ex / dur / 1e12,
           "wait_any_share": (c.get("SQ_WAIT_ANY", 0.0) / c["SQ_WAVE_CYCLES"]) if c.get("SQ_WAVE_CYCLES") else None,
           "formula": "FMA_F64 x 128 + (ADD_F64 + MUL_F64) x 64 + MFMA_MOPS_F64 x 512"}
    if units:
        rec["units_per_dispatch"] = units
        rec["unit"] = unit
        rec["executed_flops_per_unit"] = ex / units
    print(json.dumps(rec))


if __name__ == "__main__":
    main(sys.argv[1:])
