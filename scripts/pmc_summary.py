"""Per-kernel rocprofv3 counter totals from scripts/gpu_pmc.sh passes, as JSON.

    python scripts/pmc_summary.py OUT.json SAMPLES DIR [DIR ...]

Sums counter_collection.csv values per kernel name over all dispatches in each pass directory and
derives, per kernel (SAMPLES = samples of the frames the passes profiled):
  valu_insts_per_sample  SQ_INSTS_VALU / SAMPLES (wave-level instructions)
  lanes_active           SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU (active lanes per VALU issue)
  valu_busy              SQ_ACTIVE_INST_VALU x 2 cycles (a wave64 VALU op issues over 2 cycles on a
                         SIMD-32, MI355X_MICROARCH.md) / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs): the
                         share of SIMD cycles issuing VALU (GRBM_GUI_ACTIVE sums the 8 XCDs' clocks)
  lds_bank_conflict_frac SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  fetch_bytes / write_bytes  FETCH_SIZE x 2 / WRITE_SIZE in bytes (KB x 1024; FETCH doubled per
                         MI355X_MICROARCH.md: gfx950 tallies 128-B read requests at 64 B)
"""
import collections
import csv
import glob
import json
import sys


def main():
    out, samples, dirs = sys.argv[1], float(sys.argv[2]), sys.argv[3:]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"]
                agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[name].add((d, r.get("Dispatch_Id", "")))
    res = {}
    for name, c in agg.items():
        if not any(k in name for k in ("rt_book1", "rt_render", "rt_general", "chain_")):
            continue
        e = {"counters": dict(c), "dispatches_per_pass": max(1, len(disp[name]) // max(1, len(dirs)))}
        if c.get("SQ_INSTS_VALU"):
            e["valu_insts_per_sample"] = c["SQ_INSTS_VALU"] / samples
        if c.get("SQ_ACTIVE_INST_VALU"):
            e["lanes_active"] = c.get("SQ_THREAD_CYCLES_VALU", 0.0) / c["SQ_ACTIVE_INST_VALU"]
            if c.get("GRBM_GUI_ACTIVE"):
                e["valu_busy"] = c["SQ_ACTIVE_INST_VALU"] * 2 / (1024 * c["GRBM_GUI_ACTIVE"] / 8)
        if c.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_bank_conflict_frac"] = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_LDS_IDX_ACTIVE"]
        if "FETCH_SIZE" in c:
            e["fetch_bytes"] = c["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in c:
            e["write_bytes"] = c["WRITE_SIZE"] * 1024
        res[name] = e
    json.dump({"samples": samples, "passes": dirs, "kernels": res}, open(out, "w"), indent=1, sort_keys=True)
    for name, e in res.items():
        print(name, {k: (round(v, 4) if isinstance(v, float) else v) for k, v in e.items() if k != "counters"})


if __name__ == "__main__":
    main()
