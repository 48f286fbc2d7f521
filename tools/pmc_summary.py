"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/p*/run_counter_collection.csv) for one kernel.

HBM traffic per launch follows /opt/skills/guides/MI355X_MICROARCH.md (HBM section):
FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of wide
coalesced streaming reads (16 B/lane, incl. global_load_lds) -> x2; WRITE_SIZE is exact for
16 B/lane stores.  hbm_bytes_per_launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.

python tools/pmc_summary.py <pmc_dir> <kernel-substring> <algorithmic_bytes> <flops> [period:stride:phase] > out.json

The optional selector keeps, among the matching dispatches of each pass in dispatch order, ordinal o with
o % period < period - period % stride and (o % period) % stride == phase: e.g. 97:3:1 picks the attention
projections out of the ViT-H forward's 97 launches of gemm_pp_kernel<0,...> (32 x (qkv, proj, fc2) + deconv 1).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    d, key, alg_bytes, flops = sys.argv[1], sys.argv[2], float(sys.argv[3]), float(sys.argv[4])
    sel = [int(v) for v in sys.argv[5].split(":")] if len(sys.argv) > 5 else None
    csv.field_size_limit(1 << 30)
    vals = defaultdict(list)
    dur = []
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        with open(f) as fh:
            rows = [row for row in csv.DictReader(fh) if key in row["Kernel_Name"]]
        did = "Dispatch_Id" if rows and "Dispatch_Id" in rows[0] else "Correlation_Id"
        order = {k: i for i, k in enumerate(sorted({int(r[did]) for r in rows}))}
        for row in rows:
            if sel:
                period, stride, phase = sel
                r = order[int(row[did])] % period
                if r >= period - period % stride or r % stride != phase:
                    continue
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
            dur.append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    avg = {k: sum(v) / len(v) for k, v in vals.items()}
    out = {"kernel": key + (f" [dispatch selector {sys.argv[5]}]" if sel else ""), "samples": {k: len(v) for k, v in vals.items()}, "counters_avg_per_launch": avg,
           "algorithmic_bytes_per_launch": alg_bytes, "flops_per_launch": flops,
           "method": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (MI355X_MICROARCH.md HBM section gfx950 corrections)"}
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        rd, wr = 2 * avg["FETCH_SIZE"] * 1024, avg["WRITE_SIZE"] * 1024
        out.update(hbm_read_bytes_per_launch=rd, hbm_write_bytes_per_launch=wr, hbm_bytes_per_launch=rd + wr,
                   traffic_over_algorithmic=(rd + wr) / alg_bytes)
    if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
        out["l2_hit_rate"] = avg["TCC_HIT_sum"] / max(1.0, avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
    if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
        out["mfma_busy_per_gui_cycle"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / max(1.0, avg["GRBM_GUI_ACTIVE"])
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS give-back): the share of the chip's
        # 1,024 SIMD-cycles in which a matrix pipe was busy
        out["mfma_busy_fraction"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / max(1.0, avg["GRBM_GUI_ACTIVE"] / 8 * 1024)
    if "SQ_WAVE_CYCLES" in avg:
        wc = max(1.0, avg["SQ_WAVE_CYCLES"])
        out["wave_cycle_split"] = {k: avg[k] / wc for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")
                                   if k in avg}
    if dur:
        out["avg_duration_ns_under_pmc"] = sum(dur) / len(dur)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
