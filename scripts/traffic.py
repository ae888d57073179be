"""HBM traffic per launch from rocprofv3 PMC passes (MI355X_MICROARCH.md, HBM section):
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half of the bytes of 16-B-per-lane
streaming reads, so it is doubled for the kernels that read that way (STREAM16); WRITE_SIZE is taken
as is.  Writes profiles/<round>/traffic.json keyed by kernel name.

usage: python scripts/traffic.py <pmc dir with p*/run_counter_collection.csv> <out.json> "<command>"
"""
import collections
import csv
import glob
import json
import sys

root, out, cmd = sys.argv[1], sys.argv[2], sys.argv[3]
# kernels whose payload reads are 16-B-per-lane streaming loads (the calibrated case: FETCH_SIZE x2);
# every other kernel's FETCH_SIZE is reported raw (a lower bound: its access widths are uncalibrated,
# MI355X_MICROARCH.md HBM section), with the x2 figure beside it as the upper bound
STREAM16 = ("k_pair_tasks", "k_wide_reduce", "k_bsi_range", "k_bsi_chain", "k_pair_small<")
# Round 6 calibration (scripts/micro/fetch_calib.cpp, profiles/r06/calib): on known 4-GiB reads FETCH_SIZE is
# TCC_EA0_RDREQ x 64 B with TCC_BUBBLE = 0 — coalesced 8-B and 16-B per lane reads issue 128-B requests (FETCH =
# 1/2 of the bytes), scattered 16-B pieces of 64-B segments issue 64-B requests (FETCH = the bytes).  naive_xor's
# reads are its coalesced key-major records and its run lists by LDS-DMA: FETCH x 1 falls below what the kernel
# provably reads (records + payload arena, bench.py provable_min_read_bytes) and FETCH x 2 lies just above it, so
# both streams are 128-B requests and x 2 is the calibrated figure.  workShyAnd is the same case: its 16 lanes of a
# member read 16 consecutive keys' run counts, offsets and run lists — consecutive containers, whole lines — and
# raw FETCH (5.2 GB) falls below the run arena alone (6.4 GB), so its requests are 128-B lines too.
WIDE128 = ("k_wide_runs_xor", "k_wide_runs_and")
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        name = row["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        # one group per (kernel, grid): the same kernel at another problem size is another workload
        vals[(name, int(row["Grid_Size"]))][row["Counter_Name"]].append(float(row["Counter_Value"]))
res = {}
for (name, grid), c in vals.items():
    if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
        continue
    raw = 1024.0 * sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"])
    calibrated = any(k in name for k in STREAM16 + WIDE128)
    fetch = 2.0 * raw if calibrated else raw
    write = 1024.0 * sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"])
    g = {"grid": grid, "fetch_bytes": int(fetch), "write_bytes": int(write), "traffic_bytes": int(fetch + write),
         "dispatches": len(c["FETCH_SIZE"]),
         "fetch_correction": ("x2 (128-B line requests; raw < the kernel's provable reads; calibrated, profiles/r06/calib)"
                              if any(k in name for k in WIDE128) else "x2 (16-B/lane streaming reads)") if calibrated
                             else "raw (mixed or uncalibrated widths: lower bound; traffic_bytes_x2 the upper)",
         "traffic_bytes_x2": int(2.0 * raw + write)}
    res.setdefault(name, []).append(g)
for name in res:
    res[name].sort(key=lambda g: -g["traffic_bytes"])
json.dump({"command": cmd, "correction": "FETCH_SIZE KiB->B; x2 for the 16-B/lane streaming kernels only "
                                         "(per-group fetch_correction)", "kernels": res},
          open(out, "w"), indent=1, sort_keys=True)
for name, gs in res.items():
    print(name, gs[0])
