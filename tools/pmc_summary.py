"""Turn a gpurun_out/<tag>/ evidence pass (tools/gpu_profile.sh) into the committed summaries:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<tag>_pmc.json           per-launch FETCH_SIZE / WRITE_SIZE of the closed-loop kernel
  profiles/pmc_latest.json          what bench.py reads for roofline.traffic (keyed by the
                                    profiled libmpct.so's sha256)
  profiles/<tag>_bench.json         the bench line of the same pass

FETCH_SIZE / WRITE_SIZE are KiB per dispatch.  gfx950 correction (MI355X_MICROARCH.md, HBM
section): FETCH_SIZE counts 64 B per 128 B request, so the read bytes are 2 x FETCH_SIZE;
WRITE_SIZE is taken as reported.
Usage: python tools/pmc_summary.py r01 [--candidates 4096 --n2 30 --nu 5]
"""
import argparse
import csv
import json
import os
import shutil
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "gpc_small_kernel"  # the metric's timed instance (--kernel for another)


def counter(path, name):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == name]
    if not vals:
        raise SystemExit("no %s samples for %s in %s" % (name, KERNEL, path))
    return statistics.median(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--candidates", type=int, default=4096)
    ap.add_argument("--n2", type=int, default=30)
    ap.add_argument("--nu", type=int, default=5)
    ap.add_argument("--kernel", default=KERNEL)
    a = ap.parse_args()
    globals()["KERNEL"] = a.kernel
    src = os.path.join(ROOT, "gpurun_out", a.tag)
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"), os.path.join(dst, a.tag + "_kernel_stats.csv"))
    avg_ns = None
    for r in csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_stats.csv"))):
        if KERNEL in r["Name"]:
            avg_ns = float(r["AverageNs"])
    fetch_kib, nf = counter(os.path.join(src, "fetch", "fetch_counter_collection.csv"), "FETCH_SIZE")
    write_kib, nw = counter(os.path.join(src, "write", "write_counter_collection.csv"), "WRITE_SIZE")
    read_b = 2.0 * fetch_kib * 1024.0
    write_b = write_kib * 1024.0
    out = {
        "tag": a.tag, "kernel": KERNEL, "candidates": a.candidates, "n2": a.n2, "nu": a.nu,
        "kernel_avg_ns_rocprof": avg_ns,
        "fetch_size_kib_median": fetch_kib, "write_size_kib_median": write_kib,
        "dispatches": {"fetch": nf, "write": nw},
        "hbm_read_bytes_per_launch": read_b, "hbm_write_bytes_per_launch": write_b,
        "hbm_bytes_per_launch": read_b + write_b,
        "correction": "read = 2 x FETCH_SIZE (gfx950), write = WRITE_SIZE; KiB -> bytes x1024",
        # the library the counter passes profiled (tools/gpu_profile.sh records it on the box);
        # bench.py uses hbm_bytes_per_launch only when the library it loads has this hash
        "lib_sha256": open(os.path.join(src, "lib_sha256.txt")).read().split()[0],
    }
    import glob
    agg = {}
    for sub in ("sq", "sq2"):  # tools/gpu_evidence.sh: two SQ passes (8 SQ counters each)
        for f in glob.glob(os.path.join(src, sub, "*counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                if KERNEL in r["Kernel_Name"]:
                    agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    if agg:
        med = {k: statistics.median(v) for k, v in agg.items()}
        steps = a.candidates * 500.0
        out["sq"] = {"per_launch_median": med,
                     "per_sim_step": {k: med[k] / steps for k in sorted(med) if k.startswith("SQ_INSTS")
                                      or k == "SQ_WAVE_CYCLES"},
                     "lds_bank_conflict_per_lds_active": med.get("SQ_LDS_BANK_CONFLICT", 0.0) /
                     max(med.get("SQ_LDS_IDX_ACTIVE", 1.0), 1.0),
                     "note": "SQ_WAVE_CYCLES in quad-cycles (MI355X_MICROARCH.md); tools/ab.py batch"}
        f64 = ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64")
        if all(k in med for k in f64) and avg_ns:
            # every issued FP64 VALU wave-instruction counted at 64 lanes (FMA = 2 flops): the FP64
            # rate the SIMDs issued, an upper bound on lane-level FP64 work (masked lanes count)
            fl = 64.0 * (2.0 * med[f64[0]] + med[f64[1]] + med[f64[2]])
            out["fp64_counter"] = {"flops_issued_per_launch": fl,
                                   "tflops": fl / (avg_ns * 1e-9) / 1e12,
                                   "trans_f64_per_launch": med.get("SQ_INSTS_VALU_TRANS_F64"),
                                   "formula": "64 x (2 FMA_F64 + ADD_F64 + MUL_F64) / rocprof kernel time"}
    for name in (a.tag + "_pmc.json", "pmc_latest.json"):
        with open(os.path.join(dst, name), "w") as f:
            json.dump(out, f, indent=1)
    b = os.path.join(src, "bench.json")
    if os.path.exists(b):
        shutil.copy(b, os.path.join(dst, a.tag + "_bench.json"))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
