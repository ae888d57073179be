#!/usr/bin/env python3
"""Benchmark of the MI355X RoaringBitmap set-algebra path (BASELINE.json metric).

Default workload (N=1): SURVEY §8d config 2 — batched pairwise AND of 1M (filter,
posting-list) bitmap pairs with mixed Array/Bitmap/Run containers, generated on the device
(SplitMix64, seed 42 + rank).  One "step" = one rbgpu_pairwise(AND) call over every pair,
inputs already resident in HBM, results materialized in HBM (RoaringFormatSpec payloads).

Multi-GPU (torchrun, one process per GPU): pairs are independent, so each rank owns its own
1M pairs (weak scaling, no data-path collective); barrier + max-over-ranks timing.

Output: one JSON line on rank 0 with `roofline` (dominant kernel k_pairwise: algorithmic bytes
per launch / HIP-event duration on the library stream, against 8 TB/s HBM) and `cpu_baseline`
(the oracle — C++ restatement of RoaringBitmap.and — on a bounded sample, host threads).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "input GB/s (HBM roofline %) for batched and/or/xor + wide-OR, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


TRAFFIC_JSON = os.path.join(ROOT, "profiles", "r01", "traffic.json")


def pair_traffic(op, main_name):
    """PMC HBM bytes per launch of the pairwise task phase: light, heavy, or both when they run
    concurrently (the span "k_pair_tasks<light>||<heavy>")."""
    lt = pmc_traffic(f"rbg::k_pair_tasks<{op}, false, 0>", True)
    hv = pmc_traffic(f"rbg::k_pair_tasks<{op}, false, 1>", True)
    if "||" in main_name:
        # the concurrent phase launches the light kernel twice (beside the heavy kernel, then on the
        # side stream after it; one task queue): its bytes per phase = all light dispatches' bytes
        # over the number of phases (= heavy dispatches)
        if lt is None or hv is None:
            return None
        return int(lt[0] * lt[1] / max(hv[1], 1)) + hv[0]
    x = lt if "light" in main_name else hv
    return x[0] if x else None


def pmc_traffic(pmc_name: str, with_count: bool = False):
    """HBM bytes per launch of `pmc_name` from the committed rocprofv3 PMC summary of this same bench
    command (scripts/traffic.py: FETCH_SIZE x2 for gfx950 16-B/lane reads + WRITE_SIZE, separate
    passes); the dominant (largest) dispatch group is the headline launch.  None if not profiled."""
    try:
        with open(TRAFFIC_JSON) as f:
            groups = json.load(f)["kernels"].get(pmc_name)
        if not groups:
            return None
        return (int(groups[0]["traffic_bytes"]), int(groups[0]["dispatches"])) if with_count else \
            int(groups[0]["traffic_bytes"])
    except (OSError, ValueError, KeyError):
        return None


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--pairs", type=int, default=1_000_000, help="pairs per GPU (config 2)")
    p.add_argument("--workload", default="pairwise_and",
                   choices=["pairwise_and", "pairwise_or", "pairwise_xor", "pairwise_andnot", "wide_or",
                            "wide_and_runs", "wide_xor_runs"])
    p.add_argument("--wide-bitmaps", type=int, default=0, help="bitmaps of a wide workload (0: the config's)")
    p.add_argument("--secondary", default="wide_or", choices=["none", "wide_or", "wide_and_runs", "wide_xor_runs"],
                   help="key-range-sharded wide workload reported beside the headline (strong scaling)")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--census", type=int, default=1, help="also report config 1 (census1881) at N=1")
    p.add_argument("--bsi", type=int, default=1, help="also report config 5 (BSI RANGE, 64 x 100M) at N=1")
    p.add_argument("--no-cpu-baseline", action="store_true")
    return p.parse_args()


# Rehearsal knobs (not used by the driver): RBGPU_DIST_BACKEND=gloo keeps the collectives on the
# host, RBGPU_SAME_DEVICE=1 puts every rank on device 0 — together they exercise the N>1 path on a
# one-GPU box.  The production path is one rank per GPU over RCCL ("nccl").
BACKEND = os.environ.get("RBGPU_DIST_BACKEND", "nccl")


def coll_device(local: int = 0):
    import torch
    return torch.device("cuda", local) if BACKEND == "nccl" else torch.device("cpu")


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("RBGPU_SAME_DEVICE") == "1":
        local = 0
    dist = None
    if world > 1:
        import torch
        import torch.distributed as td
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if BACKEND == "nccl":
            torch.cuda.set_device(local)
        td.init_process_group(BACKEND, rank=rank, world_size=world)
        dist = td
    return world, rank, local, dist


def barrier_max(dist, value: float) -> float:
    if dist is None:
        return value
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=coll_device(torch.cuda.current_device()
                                                                       if BACKEND == "nccl" else 0))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allreduce_sum(dist, value: float) -> float:
    if dist is None:
        return value
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=coll_device(torch.cuda.current_device()
                                                                       if BACKEND == "nccl" else 0))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def barrier(dist):
    if dist is not None:
        dist.barrier()


def cpu_baseline(ctx, rb, a, b, op, seconds: float):
    """Oracle (C++ restatement of RoaringBitmap.and etc.) on a bounded sample, host threads."""
    from oracle import rbref as R
    n_total = len(a)
    sample = min(n_total, 20000)
    ra = [R.RefBitmap.deserialize(x) for x in a.serialize(0, sample)]
    rbb = [R.RefBitmap.deserialize(x) for x in b.serialize(0, sample)]
    # algorithmic input bytes of the sample, counted exactly like the device run
    tmp = ctx.pairwise(op, a, b, np.arange(sample, dtype=np.uint32), np.arange(sample, dtype=np.uint32))
    sample_bytes = ctx.stats()["input_bytes"]
    tmp.close()
    threads = min(16, os.cpu_count() or 1)
    res = {}
    for th in (1, threads):
        passes, t0 = 0, time.perf_counter()
        while True:
            R.pairwise_batch(op, ra, rbb, threads=th)
            passes += 1
            el = time.perf_counter() - t0
            if el >= seconds / 2:
                break
        res[th] = passes * sample_bytes / el / 1e9
    return {
        "value": round(res[threads], 3), "unit": "GB/s", "cores": threads, "kind": "port",
        "value_1thread": round(res[1], 3),
        "sample": f"first {sample} of the {n_total} generated pairs, looped for ~{seconds / 2:.0f}s per thread count; "
                  f"oracle/rbref.cpp RoaringBitmap.{['and', 'or', 'xor', 'andNot'][op]} (C++ restatement, -O3)",
    }


WIDE_WORKLOADS = {
    # name: (generator workload, semantics, default bitmaps, description)
    "wide_or": ("WL_WIDE_DENSE", "FAST_OR", 1024,
                "config3: FastAggregation.or of {n} dense bitmaps over the full 2^32 universe"),
    "wide_and_runs": ("WL_WIDE_RUNS", "FAST_AND", 4096,
                      "config4: FastAggregation.and (workShyAnd) of {n} run-heavy bitmaps x 65536 keys"),
    "wide_xor_runs": ("WL_WIDE_RUNS", "FAST_XOR", 4096,
                      "config4: FastAggregation.xor (naive_xor) of {n} run-heavy bitmaps x 65536 keys"),
}


def run_wide(args, name, world, rank, local, dist, ctx, rb, nbitmaps, steps, warmup):
    """Key-range-sharded wide aggregation: rank r generates and aggregates keys [lo_r, hi_r) of the
    one global dataset (strong scaling: total work fixed), then the RCCL exchange of the shard
    summaries (roaringbitmap_amd.sharding).  The synthetic data is uniform over keys, so equal key
    ranges are byte-balanced; partition_keys() does the same from rbgpu_set_key_bytes for real data."""
    from roaringbitmap_amd.sharding import ShardedWide
    wl, sem_name, _, desc = WIDE_WORKLOADS[name]
    lo, hi = (65536 * rank) // world, (65536 * (rank + 1)) // world
    a = ctx.generate_keys(getattr(rb, wl), nbitmaps, lo, hi, seed=42)
    sem = getattr(rb, sem_name)
    sw = ShardedWide(dist, rank, world, device=coll_device(local)) if dist is not None else None

    def step():
        if sw is None:
            return ctx.wide(sem, a, key_range=(lo, hi)), None
        res = sw.aggregate(ctx, sem, a, (lo, hi))
        return res.local, res

    ctx.synchronize()
    for _ in range(warmup):
        r, _ = step()
        r.close()
    kernel_ms, kernel_bytes, in_bytes, out_bytes = [], [], 0, 0
    barrier(dist)
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        r, res = step()
        st = ctx.stats()
        kernel_ms.append(st["main_kernel_ms"])
        kernel_bytes.append(st["main_kernel_bytes"])
        in_bytes += st["input_bytes"]
        out_bytes += st["output_bytes"]
        r.close()
    ctx.synchronize()
    barrier(dist)
    elapsed = barrier_max(dist, time.perf_counter() - t0)
    total_in = allreduce_sum(dist, float(in_bytes))
    k_ms = barrier_max(dist, float(np.mean(kernel_ms)))
    k_bytes = float(np.mean(kernel_bytes))
    out = {
        "workload": desc.format(n=nbitmaps),
        "value": round(total_in / elapsed / 1e9, 3), "unit": "GB/s", "n_gpus": world, "steps": steps,
        "ms_per_step": round(elapsed / steps * 1e3, 4), "scaling": "strong",
        "input_bytes_per_step": int(total_in // steps),
        "key_range_rank0": [lo, hi],
        "parallelism": f"key-range shards x{world}; RCCL all_gather of shard summaries (cardinality, "
                       f"containers, Run containers, payload bytes) per step" if world > 1 else "single GPU",
        "roofline": {"bound": "hbm", "kernel": st["main_kernel"], "traffic": pmc_traffic(
                         "rbg::k_wide_reduce<%d>" % getattr(rb, sem_name)) if world == 1 else None,
                     "achieved": round(k_bytes / (k_ms * 1e-3) / 1e9, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(k_bytes / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "kernel_ms_max_over_ranks": round(k_ms, 4), "algorithmic_bytes_per_launch_rank0": int(k_bytes)},
    }
    if res is not None:
        out["result_cardinality"] = res.cardinality
        out["result_serialized_bytes"] = res.serialized_size
    a.close()
    return out


def wide_cpu_baseline(ctx, rb, name, seconds: float):
    """The oracle's FastAggregation (C++ restatement) on keys [0, 64) of the same dataset, 1 thread."""
    from oracle import rbref as R
    wl, sem_name, n, _ = WIDE_WORKLOADS[name]
    a = ctx.generate_keys(getattr(rb, wl), n, 0, 64, seed=42)
    refs = [R.RefBitmap.deserialize(x) for x in a.serialize()]
    r = ctx.wide(getattr(rb, sem_name), a)
    sample_bytes = ctx.stats()["input_bytes"]
    r.close()
    a.close()
    sem = getattr(R, sem_name)
    passes, t0 = 0, time.perf_counter()
    while True:
        R.wide(sem, refs)
        passes += 1
        if time.perf_counter() - t0 >= seconds:
            break
    el = time.perf_counter() - t0
    return {"value": round(passes * sample_bytes / el / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"keys [0, 64) of the {n} generated bitmaps ({sample_bytes} algorithmic input bytes), "
                      f"oracle/rbref.cpp {sem_name} looped for ~{seconds:.0f}s"}


CENSUS_EXPECTED = {"AND": 23, "OR": 2007691, "XOR": 2007668, "ANDNOT": 1003836}  # RealDataBenchmark*Test.java


def load_census(name="census1881"):
    """real-roaring-dataset zip (copied under tests/golden/realdata), entries in zip order like
    ZipRealDataRetriever (real-roaring-dataset/.../ZipRealDataRetriever.java:50-67)."""
    import zipfile
    z = zipfile.ZipFile(os.path.join(ROOT, "tests", "golden", "realdata", name + ".zip"))
    out = []
    for info in z.infolist():
        txt = z.read(info).decode().strip()
        out.append(np.array([int(x) for x in txt.split(",") if x.strip()], dtype=np.uint32))
    return out


def run_census(args, ctx, rb):
    """Config 1: RealDataBenchmark{And,Or,Xor,AndNot} on census1881 — 199 consecutive pairs (k, k+1)
    of the 200 bitmaps (bitmapOf), one batched call per op; a step is the four ops."""
    vals = load_census()
    s = ctx.upload_values(vals)
    n = len(vals) - 1
    ai = np.arange(n, dtype=np.uint32)
    bi = ai + 1
    ops = {"AND": rb.AND, "OR": rb.OR, "XOR": rb.XOR, "ANDNOT": rb.ANDNOT}
    cards = {k: int(ctx.pairwise(op, s, s, ai, bi).cardinalities().sum()) for k, op in ops.items()}
    for _ in range(args.warmup):
        for op in ops.values():
            ctx.pairwise(op, s, s, ai, bi).close()
    ctx.synchronize()
    in_bytes = 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        for op in ops.values():
            ctx.pairwise(op, s, s, ai, bi).close()
            in_bytes += ctx.stats()["input_bytes"]
    ctx.synchronize()
    el = time.perf_counter() - t0
    out = {"workload": "config1: census1881 RealDataBenchmark and/or/xor/andNot, 199 consecutive pairs per op",
           "value": round(in_bytes / el / 1e9, 3), "unit": "GB/s", "ms_per_step": round(el / args.steps * 1e3, 4),
           "us_per_op_sweep": round(el / args.steps / 4 * 1e6, 1), "cardinality_sums": cards,
           "golden_ok": cards == CENSUS_EXPECTED}
    if not args.no_cpu_baseline:
        from oracle import rbref as R
        refs = [R.RefBitmap.deserialize(x) for x in s.serialize()]
        a_r, b_r = refs[:-1], refs[1:]
        passes, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < 2.0:
            for op in ops.values():
                R.pairwise_batch(op, a_r, b_r, threads=1)
            passes += 1
        el = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(passes * in_bytes / args.steps / el / 1e9, 3), "unit": "GB/s",
                               "cores": 1, "kind": "port", "us_per_op_sweep": round(el / passes / 4 * 1e6, 1),
                               "sample": "the whole config (199 pairs x 4 ops), oracle/rbref.cpp, 1 thread"}
    s.close()
    return out


def run_bsi(args, ctx, rb, nslices=64, nrows=100_000_000, steps=5, warmup=2):
    """Config 5: Roaring64BitmapSliceIndex.compare(RANGE, lo, hi, null) over 64 slices x 100M rows
    (runOptimize'd BSI, random value bits) — one fused pass per high key for each O'Neil chain."""
    d = ctx.generate_bsi(nslices, nrows, seed=42)
    lo, hi = 0x3A00_0000_0000_0000, 0xB100_0000_0000_0000  # a mid-range window: no min/max shortcut
    vmin, vmax = 0, (1 << nslices) - 1
    for _ in range(warmup):
        ctx.bsi_compare(rb.BSI_RANGE, d, lo, hi, vmin, vmax).close()
    ctx.synchronize()
    in_bytes, k_ms, k_bytes = 0, [], []
    t0 = time.perf_counter()
    for _ in range(steps):
        r = ctx.bsi_compare(rb.BSI_RANGE, d, lo, hi, vmin, vmax)
        st = ctx.stats()
        in_bytes += st["input_bytes"]
        k_ms.append(st["main_kernel_ms"])
        k_bytes.append(st["main_kernel_bytes"])
        card = None
        if _ == steps - 1:
            card = int(r.cardinalities()[0])
        r.close()
    ctx.synchronize()
    el = time.perf_counter() - t0
    km, kb = float(np.mean(k_ms)), float(np.mean(k_bytes))
    out = {"workload": f"config5: BSI compare RANGE over {nslices} slices x {nrows} rows (2 O'Neil chains + AND, "
                       "fused into one pass per key)",
           "value": round(in_bytes / el / 1e9, 3), "unit": "GB/s", "ms_per_step": round(el / steps * 1e3, 4),
           "result_cardinality": card,
           "roofline": {"bound": "hbm", "kernel": st["main_kernel"],
                        "traffic": pmc_traffic("rbg::k_bsi_range"),
                        "note": "the fused kernel reads every slice container once for both comparators "
                                "(GE and LE); algorithmic bytes count that one read",
                        "achieved": round(kb / (km * 1e-3) / 1e9, 2),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(kb / (km * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        "kernel_ms": round(km, 4), "algorithmic_bytes_per_launch": int(kb)}}
    if not args.no_cpu_baseline:
        from oracle import rbref as R
        small = ctx.generate_bsi(nslices, 4 * 65536, seed=42)  # the first 4 keys of the same shape
        refs = [R.RefBitmap.deserialize(x) for x in small.serialize()]
        r = ctx.bsi_compare(rb.BSI_RANGE, small, lo, hi, vmin, vmax)
        sb = ctx.stats()["input_bytes"]
        r.close()
        small.close()
        passes, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < 3.0:
            R.bsi_compare(refs[:-1], refs[-1], R.BSI_RANGE, lo, hi, None, vmin, vmax)
            passes += 1
        el = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(passes * sb / el / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": "port",
                               "sample": f"the same query on 4 x 65536 rows ({sb} algorithmic input bytes), "
                                         "oracle/rbref.py BSI restatement over rbref.cpp static ops, 1 thread"}
    d.close()
    return out


def main():
    args = parse()
    world, rank, local, dist = dist_setup(args)
    import roaringbitmap_amd as rb
    ctx = rb.Context(local)
    seed = 42 + rank

    if args.workload in WIDE_WORKLOADS:
        nb = args.wide_bitmaps or WIDE_WORKLOADS[args.workload][2]
        w = run_wide(args, args.workload, world, rank, local, dist, ctx, rb, nb, args.steps, args.warmup)
        if rank == 0:
            line = {"metric": METRIC, "value": w["value"], "unit": "GB/s", "n_gpus": world, "steps": args.steps,
                    "warmup": args.warmup, "ms_per_step": w["ms_per_step"], "higher_is_better": True,
                    "scaling": "strong", "vs_baseline": None, "dtype": "u64",
                    "data": "synthetic (device SplitMix64 generator keyed by (bitmap, key); SURVEY §8d)",
                    "config": {k: v for k, v in w.items() if k not in ("value", "roofline", "ms_per_step")},
                    "roofline": w["roofline"]}
            if world == 1 and not args.no_cpu_baseline:
                line["cpu_baseline"] = wide_cpu_baseline(ctx, rb, args.workload, args.cpu_seconds / 2)
            print(json.dumps(line), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return

    op = {"pairwise_and": rb.AND, "pairwise_or": rb.OR, "pairwise_xor": rb.XOR, "pairwise_andnot": rb.ANDNOT}[
        args.workload]
    a, b = ctx.generate(rb.WL_FILTER_POSTING, args.pairs, seed=seed)
    run = lambda: ctx.pairwise(op, a, b)  # noqa: E731
    workload = (f"config2: batched pairwise {['AND', 'OR', 'XOR', 'ANDNOT'][op]} of {args.pairs} "
                f"(filter, posting-list) pairs per GPU, mixed Array/Bitmap/Run, 2^18 universe")
    units = args.pairs
    unit_name = "pairs"
    ctx.synchronize()

    for _ in range(args.warmup):
        r = run()
        r.close()
    ctx.synchronize()

    kernel_ms, kernel_bytes, in_bytes, out_bytes = [], [], 0, 0
    per_kernel = {}
    barrier(dist)
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r = run()
        st = ctx.stats()
        kernel_ms.append(st["main_kernel_ms"])
        kernel_bytes.append(st["main_kernel_bytes"])
        for k in st["kernels"]:
            agg = per_kernel.setdefault(k["name"], {"ms": 0.0, "bytes": 0, "items": 0})
            agg["ms"] += k["ms"] / args.steps
            agg["bytes"] += k["bytes"] // args.steps
            agg["items"] += k["items"] // args.steps
        in_bytes += st["input_bytes"]
        out_bytes += st["output_bytes"]
        r.close()
    ctx.synchronize()
    barrier(dist)
    elapsed = time.perf_counter() - t0
    elapsed = barrier_max(dist, elapsed)
    total_in = allreduce_sum(dist, float(in_bytes))
    total_out = allreduce_sum(dist, float(out_bytes))  # every rank joins every collective
    main_name = st["main_kernel"]

    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = total_in / elapsed / 1e9
        per_launch = float(np.mean(kernel_bytes))
        k_ms = float(np.mean(kernel_ms))
        achieved = per_launch / (k_ms * 1e-3) / 1e9
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (device SplitMix64 generator, runOptimize'd containers; SURVEY §8d)",
            "config": {
                "workload": workload,
                "units_per_gpu": units,
                "unit": unit_name,
                "input_bytes_per_step_per_gpu": in_bytes // args.steps,
                "output_bytes_per_step_per_gpu": out_bytes // args.steps,
                "roofline_pct_whole_step": round(100.0 * (total_in + total_out) / elapsed / 1e9 / (HBM_PEAK_GBS * world),
                                                 2),
                "parallelism": f"key-range/pair sharding x{world} (replicas, no data-path collective)",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": main_name,
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": pair_traffic(op, main_name),
                "traffic_source": "profiles/r01/traffic.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes)",
                "kernel_ms": round(k_ms, 4),
                "algorithmic_bytes_per_launch": int(per_launch),
                "kernels": {n: {"ms": round(v["ms"], 4), "bytes": v["bytes"], "items": v["items"],
                                "GB/s": round(v["bytes"] / max(v["ms"], 1e-9) / 1e6, 1)}
                            for n, v in per_kernel.items()},
            },
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(ctx, rb, a, b, op, args.cpu_seconds)
    if args.secondary != "none" or (world == 1 and (args.census or args.bsi)):
        a.close()
        b.close()
    if world == 1 and args.census:
        c1 = run_census(args, ctx, rb)
        if rank == 0:
            line.setdefault("secondary", {})["census1881"] = c1
    if world == 1 and args.bsi:
        line.setdefault("secondary", {})["bsi_range"] = run_bsi(args, ctx, rb)
    if args.secondary != "none":
        w = run_wide(args, args.secondary, world, rank, local, dist, ctx, rb,
                     WIDE_WORKLOADS[args.secondary][2], max(3, args.steps // 3), 1)
        if rank == 0:
            if world == 1 and not args.no_cpu_baseline:
                w["cpu_baseline"] = wide_cpu_baseline(ctx, rb, args.secondary, args.cpu_seconds / 2)
            line.setdefault("secondary", {})[args.secondary] = w
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
