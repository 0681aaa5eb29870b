"""Summarise a rocprofv3 SQ VALU pass into profiles/valu_counts.json (the counter
backing of bench.py's roofline.frac).

    python tools/pmc_valu.py <key> <pmc_dir> <walker_steps_per_launch> [out.json]

The pass (tools/pmc_valu.sh) collects SQ_INSTS_VALU and the FP64 VALU mix
(SQ_INSTS_VALU_FMA_F64 / MUL_F64 / ADD_F64 / TRANS_F64) of the sampler kernel: wave-level
instruction counts per dispatch, averaged over the olpe_gibbs_kernel dispatches and
divided by the walker-steps of one launch.  A wave64 FP64 instruction is 64 lane-ops,
so executed FP64 lane-ops per walker-step = 64 x (FMA + MUL + ADD + TRANS).  The entry
records the kernel digest (olpefit_amd.build.kernel_digest) it was measured on; bench.py
marks the counts stale when the library has changed since.
"""
import csv
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
COUNTERS = ("SQ_INSTS_VALU", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64",
            "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64")


def main():
    from olpefit_amd.build import kernel_digest
    key, d, steps = sys.argv[1], sys.argv[2], float(sys.argv[3])
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(REPO, "profiles", "valu_counts.json")
    acc = {c: [] for c in COUNTERS}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if "olpe_gibbs_kernel" in r["Kernel_Name"] and r["Counter_Name"] in acc:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    per = {c: sum(v) / len(v) / steps for c, v in acc.items()}
    fp64 = sum(per[c] for c in COUNTERS[1:])
    data = json.load(open(out)) if os.path.exists(out) else {}
    data[key] = {
        "valu_per_step": per["SQ_INSTS_VALU"],
        "fp64_per_step": fp64,
        "fp64_lane_ops_per_step": 64 * fp64,
        "mix_per_step": {c.replace("SQ_INSTS_VALU_", ""): per[c] for c in COUNTERS[1:]},
        "dispatches": len(acc["SQ_INSTS_VALU"]),
        "walker_steps_per_launch": steps,
        "kernel_digest": kernel_digest(),
        "source": f"rocprofv3 --pmc {' '.join(COUNTERS)} ({d})",
    }
    json.dump(data, open(out, "w"), indent=1)
    print(key, json.dumps(data[key]))


if __name__ == "__main__":
    main()
