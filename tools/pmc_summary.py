"""Summarise the rocprofv3 --pmc passes of scripts/pmc.sh into per-kernel medians and the
HBM traffic per launch that bench.py's roofline reports.

FETCH_SIZE / WRITE_SIZE are in KB per dispatch; on gfx950 FETCH_SIZE reports half the
bytes of a wide coalesced read, so it is doubled (MI355X_MICROARCH.md §HBM).  Both count
Infinity-Cache hits, so the figure is fabric traffic below L2, an upper bound on HBM.

The summary records the library the passes profiled: the "build" object of the bench JSON line
each pass printed (swarm_build_info() with its source digest, and the .so's sha256).  Every pass
must name the same build; bench.py uses a summary's counters only for that build.

usage: python tools/pmc_summary.py gpurun_out/pmc profiles/r04_pmc_tick.json
"""
import collections
import csv
import glob
import json
import os
import statistics
import sys

# "rollout": the acting-only line's kernel, the kNN + GAT specialised rollout of GoTo 8 x 1024 with
# k = 5 (bench.py --mode act --graph knn --knn-k 5; the headline acting_only line)
KERNELS = {"tick": "tick_kernel", "td": "td_kernel", "act": "act_kernel<8, 1>", "reduce": "grad_reduce_kernel",
           "rollout": "act_kernel<8, 2, 0, 3, 0>"}


def pass_builds(src):
    """The "build" object of the bench line in every pass log (p1.log, p2.log, ...)."""
    builds = {}
    for f in sorted(glob.glob(os.path.join(src, "p*.log"))):
        for line in open(f, errors="replace"):
            line = line.strip()
            if line.startswith("{") and '"build"' in line:
                try:
                    builds[os.path.basename(f)] = json.loads(line)["build"]
                except (ValueError, KeyError):
                    pass
    return builds


def main(src, dst):
    builds = pass_builds(src)
    distinct = {json.dumps(b, sort_keys=True) for b in builds.values()}
    if len(distinct) != 1:
        raise SystemExit(f"pass logs name {len(distinct)} builds (need exactly one): {builds}")
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(src, "p*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            for key, pat in KERNELS.items():
                if pat in r["Kernel_Name"]:
                    vals[(key, r["Counter_Name"])].append(float(r["Counter_Value"]))
    out = {"source": "rocprofv3 --kernel-trace --pmc, separate passes (scripts/pmc.sh), bench.py workload",
           "units": "counter medians per dispatch; *_bytes in bytes",
           "build": next(iter(builds.values())), "passes": sorted(builds),
           "kernels": {}}
    for key in KERNELS:
        k = {c: statistics.median(v) for (kk, c), v in vals.items() if kk == key}
        if not k:
            continue
        fetch = 2.0 * k.get("FETCH_SIZE", 0.0) * 1024.0
        write = k.get("WRITE_SIZE", 0.0) * 1024.0
        waves = k.get("SQ_WAVES", 0.0) or 1.0
        out["kernels"][key] = {
            "counters": k,
            "fetch_bytes_corrected": fetch,
            "write_bytes": write,
            "hbm_bytes_per_launch": fetch + write,
            "per_wave": {c: k[c] / waves for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_MFMA",
                                                    "SQ_WAVE_CYCLES", "SQ_WAIT_ANY") if c in k},
        }
        if "SQ_VALU_MFMA_BUSY_CYCLES" in k and k.get("GRBM_GUI_ACTIVE"):
            # MFMA pipe cycles over every SIMD's cycles while the GPU was busy with the dispatch:
            # GRBM_GUI_ACTIVE sums the 8 XCDs, each with 128 SIMDs (reads high on short dispatches)
            out["kernels"][key]["mfma_busy_frac_grbm"] = k["SQ_VALU_MFMA_BUSY_CYCLES"] / (128.0 * k["GRBM_GUI_ACTIVE"])
    # the bench line's dominant kernel: training lines the tick (or TD) kernel, acting lines the rollout
    main_k = next((k for k in ("tick", "td", "rollout") if k in out["kernels"]), "td")
    if main_k in out["kernels"]:
        out["kernel"] = main_k
        out["hbm_bytes_per_launch"] = out["kernels"][main_k]["hbm_bytes_per_launch"]
    json.dump(out, open(dst, "w"), indent=1)
    for key, v in out["kernels"].items():
        print(f"{key:7s} fetch {v['fetch_bytes_corrected'] / 1e3:8.1f} KB  write {v['write_bytes'] / 1e3:8.1f} KB  "
              f"per wave: " + ", ".join(f"{c.replace('SQ_', '')} {x:.0f}" for c, x in v["per_wave"].items()))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc", sys.argv[2] if len(sys.argv) > 2 else
         "profiles/r01_pmc_td.json")
