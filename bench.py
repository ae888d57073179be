#!/usr/bin/env python3
"""Benchmark of the MI355X RoaringBitmap set-algebra path (BASELINE.json metric).

Headline (N=1): SURVEY §8d config 2 — batched pairwise AND of 1M (filter, posting-list) bitmap
pairs with mixed Array/Bitmap/Run containers, generated on the device (SplitMix64, seed 42 + rank).
One "step" = one rbgpu_pairwise(AND) call over every pair, inputs already resident in HBM, results
materialized in HBM (RoaringFormatSpec payloads).

Secondary lines (same JSON object, key "secondary"): config 2 at the same scale for OR / XOR /
ANDNOT; config 1 (census1881, 4 ops); config 5 (BSI RANGE, 64 x 100M); config 3 (FastAggregation.or
of 1024 dense bitmaps); config 4 (FastAggregation.and / .xor of 4096 run-heavy bitmaps).  Each
carries `roofline` (its dominant kernel's algorithmic bytes / HIP-event duration on the library
stream, against 8 TB/s, plus the PMC-measured HBM traffic of the same launch from
profiles/<round>/traffic.json) and a `cpu_baseline` with 1-thread and all-core values.

Multi-GPU (torchrun, one process per GPU):
  * pairwise (configs 2): pairs are independent, each rank owns its own 1M pairs (weak scaling);
    per step one all_reduce of the result cardinality (ShardedPairwise's exchange);
  * wide (configs 3, 4) and BSI (config 5): rank r owns a high-key range of the one global dataset
    (strong scaling), per step an all_gather of the shard summaries (global cardinality and
    serialized size: ShardedWide / ShardedBsi);
barrier + max-over-ranks timing; value = all ranks' input bytes / that time.
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
OPS = ["AND", "OR", "XOR", "ANDNOT"]


def _traffic_json():
    for rnd in ("r06", "r05", "r03", "r02", "r01"):
        p = os.path.join(ROOT, "profiles", rnd, "traffic.json")
        if os.path.exists(p):
            return p
    return None


TRAFFIC_JSON = _traffic_json()


def _traffic_groups(pmc_name):
    if TRAFFIC_JSON is None:
        return None
    try:
        with open(TRAFFIC_JSON) as f:
            kernels = json.load(f)["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    if pmc_name in kernels:
        return kernels[pmc_name] or None
    # a template instance of the named kernel (e.g. rbg::k_wide_runs_and<16>)
    hits = [g for k, g in kernels.items() if k.startswith(pmc_name + "<")]
    return hits[0] if len(hits) == 1 else None


def pmc_traffic(pmc_name: str, with_count: bool = False):
    """HBM bytes per launch of `pmc_name` from the committed rocprofv3 PMC summary of this same bench
    command (scripts/traffic.py: FETCH_SIZE x2 for gfx950 16-B/lane reads + WRITE_SIZE, separate
    passes); the dominant (largest) dispatch group is the headline launch.  None if not profiled.
    "a+b": the kernels of one timed span (e.g. naive_xor's record pre-pass and its kernel), summed."""
    if "+" in pmc_name and not with_count:
        parts = [pmc_traffic(x) for x in pmc_name.split("+")]
        return None if any(x is None for x in parts) else sum(parts)
    g = _traffic_groups(pmc_name)
    if not g:
        return None
    return (int(g[0]["traffic_bytes"]), int(g[0]["dispatches"])) if with_count else int(g[0]["traffic_bytes"])


def pair_traffic(op, main_name):
    """PMC HBM bytes per launch of the pairwise task phase: light, heavy, or both when they run
    concurrently (the span "k_pair_tasks<light>||<heavy>")."""
    lt = pmc_traffic(f"rbg::k_pair_tasks<{op}, false, 0>", True)
    hv = pmc_traffic(f"rbg::k_pair_tasks<{op}, false, 1>", True)
    if "||" in main_name:
        # the concurrent phase launches each kernel twice (light beside heavy, then each kind again
        # once the other has drained; one task queue per kind), so a phase's bytes are all dispatches'
        # bytes over half the light dispatch count
        if lt is None or hv is None:
            return None
        phases = max(lt[1] // 2, 1)
        return int((lt[0] * lt[1] + hv[0] * hv[1]) / phases)
    x = lt if "light" in main_name else hv
    return x[0] if x else None


def traffic_source():
    return os.path.relpath(TRAFFIC_JSON, ROOT) + " (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes)" \
        if TRAFFIC_JSON else None


# ------------------------------------------------------------------------------- host cores
def host_cores() -> dict:
    """CPUs this process may run on (affinity mask) and the cgroup CPU quota, beside the machine's
    count: the all-core CPU baseline runs one thread per schedulable CPU."""
    machine = os.cpu_count() or 1
    try:
        sched = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        sched = machine
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(p)
    except (OSError, ValueError):
        pass
    return {"machine_cpus": machine, "schedulable_cpus": sched, "cgroup_cpu_quota": quota}


HOST = host_cores()
ALL_CORES = HOST["schedulable_cpus"]
# thread counts the all-core baselines try: every schedulable CPU, and the cgroup's CPU share when
# it is smaller (more threads than the quota only time-share it); the best is `value`
THREAD_COUNTS = sorted({ALL_CORES} | ({max(1, int(HOST["cgroup_cpu_quota"]))}
                                      if HOST["cgroup_cpu_quota"] and HOST["cgroup_cpu_quota"] < ALL_CORES else set()))


def time_loop(fn, seconds: float):
    """Passes per second of fn, looping for at least `seconds` (at least one pass)."""
    passes, t0 = 0, time.perf_counter()
    while True:
        fn()
        passes += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            return passes / el


def multi_rate(fn_threads, seconds: float):
    """{threads: passes/s} of fn_threads(threads) for 1 and THREAD_COUNTS, `seconds` split evenly."""
    counts = [1] + [t for t in THREAD_COUNTS if t > 1]
    return {t: time_loop(lambda: fn_threads(t), seconds / len(counts)) for t in counts}


def baseline_entry(bytes_per_pass, rates: dict, kind, sample, extra=None):
    """`value` = the best thread count's rate (the CPU at its best on this workload), with every
    measured count beside it."""
    best = max(rates, key=lambda t: rates[t])
    # cores = the CPUs those threads actually had: above the cgroup quota, threads only time-share it
    quota = HOST["cgroup_cpu_quota"]
    cores = min(best, max(1, int(quota))) if quota else min(best, ALL_CORES)
    out = {"value": round(bytes_per_pass * rates[best] / 1e9, 3), "unit": "GB/s", "cores": cores, "threads": best,
           "kind": kind,
           "value_1thread": round(bytes_per_pass * rates[1] / 1e9, 3),
           "by_threads": {str(t): round(bytes_per_pass * r / 1e9, 3) for t, r in rates.items()},
           "host": HOST, "sample": sample}
    if extra:
        out.update(extra)
    return out


# ------------------------------------------------------------------------------- args / dist
def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--pairs", type=int, default=1_000_000, help="pairs per GPU (config 2)")
    p.add_argument("--workload", default="pairwise_and",
                   choices=["pairwise_and", "pairwise_or", "pairwise_xor", "pairwise_andnot", "wide_or",
                            "wide_and_runs", "wide_xor_runs", "bsi_range"])
    p.add_argument("--wide-bitmaps", type=int, default=0, help="bitmaps of a wide workload (0: the config's)")
    p.add_argument("--secondary", default="all",
                   help="comma list of secondary lines: pairwise_ops,census,bsi_range,wide_or,wide_and_runs,"
                        "wide_xor_runs; 'all' or 'none'")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="headline CPU baseline budget")
    p.add_argument("--no-cpu-baseline", action="store_true")
    return p.parse_args()


SECONDARY_ALL = ["pairwise_async", "pairwise_ops", "census", "bsi_range", "wide_or", "wide_and_runs", "wide_xor_runs"]

# Rehearsal knobs (not used by the driver): RBGPU_DIST_BACKEND=gloo keeps the collectives on the
# host, RBGPU_SAME_DEVICE=1 puts every rank on device 0 — together they exercise the N>1 path on a
# one-GPU box.  The production path is one rank per GPU over RCCL ("nccl").
BACKEND = os.environ.get("RBGPU_DIST_BACKEND", "nccl")
# At N > 1 the shard exchange runs inside librbgpu on its own RCCL communicator (rbgpu_comm_*, what a Java
# caller binds), its 128-byte id handed over through torch.distributed's store before any GPU work;
# torch.distributed keeps only the barrier and the max-over-ranks timing.  RBGPU_BENCH_COMM=torch
# selects the Python exchange (sharding.py) instead — the rehearsal on one GPU needs it (RCCL refuses
# two ranks on one device).
COMM = os.environ.get("RBGPU_BENCH_COMM", "torch" if os.environ.get("RBGPU_SAME_DEVICE") == "1" else "rccl")


def coll_device(local: int = 0):
    import torch
    return torch.device("cuda", local) if BACKEND == "nccl" else torch.device("cpu")


class Dist:
    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        if os.environ.get("RBGPU_SAME_DEVICE") == "1":
            self.local = 0
        self.td = None
        if self.world > 1:
            import torch
            import torch.distributed as td
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if BACKEND == "nccl":
                torch.cuda.set_device(self.local)
            td.init_process_group(BACKEND, rank=self.rank, world_size=self.world)
            self.td = td
        self.comm, self.uid, self.comm_error = None, None, None
        self.last_step_ms = []
        if self.world == 1 and COMM == "rccl1":  # a one-rank communicator: the C-ABI exchange path at N = 1
            from roaringbitmap_amd.engine import Comm
            self.uid = Comm.unique_id()
        if self.world > 1 and COMM == "rccl":
            # the communicator id from rank 0 through the rendezvous store (no GPU touched yet)
            from roaringbitmap_amd.engine import Comm
            store = self.td.distributed_c10d._get_default_store()
            if self.rank == 0:
                try:
                    uid = Comm.unique_id().hex()
                except Exception as e:  # no RCCL id: every rank takes the torch.distributed exchange
                    uid = ""
                    self.comm_error = f"{type(e).__name__}: {e}"
                    print(f"[bench] rbgpu_comm_unique_id failed ({self.comm_error}); "
                          "the torch.distributed exchange takes over", file=sys.stderr, flush=True)
                store.set("rbgpu_comm_id", uid)
            v = store.get("rbgpu_comm_id").decode()
            self.uid = bytes.fromhex(v) if v else None

    def open_comm(self, ctx):
        """librbgpu's RCCL communicator on this rank's GPU (rbgpu_comm_init), once the context exists."""
        if self.uid is not None and self.comm is None:
            from roaringbitmap_amd.engine import Comm
            try:
                self.comm = Comm(ctx, self.uid, self.world, self.rank)
            except Exception as e:  # the line records it; the torch.distributed exchange takes over
                self.comm_error = f"{type(e).__name__}: {e}"
                print(f"[bench] rank {self.rank}: rbgpu_comm_init failed ({self.comm_error}); "
                      "falling back to the torch.distributed exchange", file=sys.stderr, flush=True)
            ok = self.reduce([1.0 if self.comm is not None else 0.0], "sum")[0] if self.td is not None else 1.0
            if self.comm is not None and ok < self.world:  # every rank uses the same path
                self.comm.close()
                self.comm = None
        return self.comm

    @property
    def device(self):
        return coll_device(self.local) if self.td is not None else None

    def barrier(self):
        if self.td is not None:
            self.td.barrier()

    def reduce(self, values, op="sum"):
        if self.td is None:
            return list(values)
        import torch
        t = torch.tensor(list(values), dtype=torch.float64, device=self.device)
        self.td.all_reduce(t, op=self.td.ReduceOp.MAX if op == "max" else self.td.ReduceOp.SUM)
        return t.cpu().tolist()

    def close(self):
        if self.comm is not None:
            self.comm.close()
        if self.td is not None:
            self.td.destroy_process_group()


def timed(D, ctx, steps, warmup, step):
    """W untimed steps, then K timed ones between barrier + device sync on both sides; returns
    (max-over-ranks elapsed, per-step stats of this rank)."""
    for _ in range(warmup):
        step()
    ctx.synchronize()
    D.barrier()
    ctx.synchronize()
    sts = []
    t0 = time.perf_counter()
    marks = [t0]
    for _ in range(steps):
        sts.append(step())
        marks.append(time.perf_counter())
    ctx.synchronize()
    D.barrier()
    el = D.reduce([time.perf_counter() - t0], "max")[0]
    # per-step wall times of this rank (a step returns once its results are in HBM: the call reads the
    # result counts back), for the spread a single mean hides
    D.last_step_ms = [1e3 * (b - a) for a, b in zip(marks, marks[1:])]
    return el, sts


def step_spread(D):
    """min / median / max of the last timed loop's per-step wall times (rank 0's)."""
    v = sorted(D.last_step_ms)
    if not v:
        return None
    return {"min": round(v[0], 4), "median": round(float(np.median(v)), 4), "max": round(v[-1], 4),
            "spread_pct": round(100.0 * (v[-1] - v[0]) / float(np.median(v)), 2)}


def roofline(main_name, k_ms, k_bytes, traffic, D, extra=None):
    k_ms_max = D.reduce([k_ms], "max")[0]
    achieved = k_bytes / (k_ms_max * 1e-3) / 1e9 if k_ms_max > 0 else 0.0
    out = {"bound": "hbm", "kernel": main_name, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
           "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
           "traffic": traffic if D.world == 1 else None, "traffic_source": traffic_source(),
           "kernel_ms": round(k_ms_max, 4), "algorithmic_bytes_per_launch": int(k_bytes)}
    if extra:
        out.update(extra)
    return out


# ------------------------------------------------------------------------------- config 2
def pairwise_line(D, ctx, rb, a, b, op, steps, warmup, npairs):
    """Config 2 for one op: every rank runs its own npairs pairs (weak scaling); per step the
    ShardedPairwise exchange (all_reduce of result cardinality / containers / bytes) at N > 1."""
    from roaringbitmap_amd.sharding import PairShardResult, ShardedPairwise
    comm = D.comm
    sp = ShardedPairwise(D.td, D.rank, D.world, D.device) if D.td is not None and comm is None else None

    def step():
        r = ctx.pairwise(op, a, b)
        st = ctx.stats_raw()  # the struct; converted to a dict after the timed loop
        glob = None
        if comm is not None or sp is not None:
            payload = st.output_bytes - 16 * st.result_containers
            if comm is not None:  # rbgpu_comm_allreduce_sum: the batch's global cardinality / containers / bytes
                g = comm.allreduce_sum([st.result_cardinality, st.result_containers, payload])
                glob = PairShardResult(None, (0, npairs), int(g[0]), int(g[1]), int(g[2]))
            else:
                glob = sp.finish(None, (0, npairs), st.result_cardinality, st.result_containers, payload)
        r.close()
        return st, glob

    from roaringbitmap_amd.engine import stats_dict
    el, sts = timed(D, ctx, steps, warmup, step)
    sts = [(stats_dict(s), g) for s, g in sts]
    in_b, out_b = sum(s["input_bytes"] for s, _ in sts), sum(s["output_bytes"] for s, _ in sts)
    ops_n = sum(s["tasks"] for s, _ in sts)
    tot_in, tot_out, tot_ops = D.reduce([float(in_b), float(out_b), float(ops_n)])
    last, glob = sts[-1]
    per_kernel = {}
    for s, _ in sts:
        for k in s["kernels"]:
            agg = per_kernel.setdefault(k["name"], {"ms": 0.0, "bytes": 0, "items": 0})
            agg["ms"] += k["ms"] / steps
            agg["bytes"] += k["bytes"] // steps
            agg["items"] += k["items"] // steps
    k_ms = float(np.mean([s["main_kernel_ms"] for s, _ in sts]))
    k_bytes = float(np.mean([s["main_kernel_bytes"] for s, _ in sts]))
    card = glob.cardinality if glob is not None else int(last["result_cardinality"])
    rl = roofline(last["main_kernel"], k_ms, k_bytes, pair_traffic(op, last["main_kernel"]), D, {
        "kernels": {n: {"ms": round(v["ms"], 4), "bytes": v["bytes"], "items": v["items"],
                        "GB/s": round(v["bytes"] / max(v["ms"], 1e-9) / 1e6, 1)} for n, v in per_kernel.items()}})
    return {
        "workload": f"config2: batched pairwise {OPS[op]} of {npairs} (filter, posting-list) pairs per GPU, "
                    f"mixed Array/Bitmap/Run, 2^18 universe",
        "value": round(tot_in / el / 1e9, 3), "unit": "GB/s", "n_gpus": D.world, "steps": steps,
        "ms_per_step": round(el / steps * 1e3, 4), "step_ms": step_spread(D), "scaling": "weak",
        "container_ops_per_s": round(tot_ops / el, 1),
        "container_ops_unit": "container-level ops per step, all ranks: matched container pairs + unmatched "
                              "containers the op copies (RoaringArray.appendCopy), each producing one result",
        "input_bytes_per_step_per_gpu": in_b // steps, "output_bytes_per_step_per_gpu": out_b // steps,
        "roofline_pct_whole_step": round(100.0 * (tot_in + tot_out) / el / 1e9 / (HBM_PEAK_GBS * D.world), 2),
        "result_cardinality_all_ranks": card, "result_containers_rank0": int(last["result_containers"]),
        "parallelism": (f"pair shards x{D.world}: each rank owns its own {npairs} pairs (no data-path collective); "
                        "per step one all_reduce of (result cardinality, containers, bytes) over "
                        + ("librbgpu's RCCL communicator (rbgpu_comm_allreduce_sum)" if comm is not None
                           else "torch.distributed")) if D.world > 1 else "single GPU",
        "roofline": rl,
    }


def pairwise_async_line(D, ctx, rb, a, b, op, steps, warmup, in_bytes, out_bytes, kernel_bytes):
    """Config 2 through rbgpu_pairwise_async: each step enqueues the next batch while the previous one
    runs (the host's per-call work and the device-to-host wait of a synchronous call leave the device's
    critical path); a step's result is freed (after it completes) one step later.  Bytes per step are the
    synchronous line's (the same pairs and results)."""
    def run(n):
        prev = None
        for _ in range(n):
            r = ctx.pairwise_async(op, a, b)
            if prev is not None:
                prev.close()
            prev = r
        if prev is not None:
            prev.wait().close()
    run(warmup)
    ctx.synchronize()
    D.barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    run(steps)
    ctx.synchronize()
    D.barrier()
    el = D.reduce([time.perf_counter() - t0], "max")[0]
    tot_in, tot_all = D.reduce([float(in_bytes * steps), float((in_bytes + out_bytes) * steps)])
    return {"workload": f"config2 {OPS[op]} as the synchronous line, batches enqueued back to back "
                        "(rbgpu_pairwise_async)",
            "value": round(tot_in / el / 1e9, 3), "unit": "GB/s", "n_gpus": D.world, "steps": steps,
            "ms_per_step": round(el / steps * 1e3, 4), "scaling": "weak",
            "roofline_pct_whole_step": round(100.0 * tot_all / el / 1e9 / (HBM_PEAK_GBS * D.world), 2),
            "note": "whole-step only: the per-kernel roofline is the synchronous line's (same kernels)"}


def pairwise_cpu_baseline(ctx, a, b, op, seconds: float, sample: int = 50000):
    """Oracle (C++ restatement of RoaringBitmap.and/or/xor/andNot) on a bounded sample of the same
    pairs: 1 thread, then one thread per schedulable host CPU (pair-parallel)."""
    from oracle import rbref as R
    n_total = len(a)
    sample = min(n_total, sample)
    ra = [R.RefBitmap.deserialize(x) for x in a.serialize(0, sample)]
    rbb = [R.RefBitmap.deserialize(x) for x in b.serialize(0, sample)]
    idx = np.arange(sample, dtype=np.uint32)
    tmp = ctx.pairwise(op, a, b, idx, idx)
    sample_bytes = ctx.stats()["input_bytes"]  # algorithmic input bytes, counted like the device run
    tmp.close()
    rates = multi_rate(lambda th: R.pairwise_batch(op, ra, rbb, threads=th), seconds)
    return baseline_entry(sample_bytes, rates, "port",
                          f"first {sample} of the {n_total} generated pairs ({sample_bytes} algorithmic input "
                          f"bytes), looped ~{seconds / len(rates):.1f}s per thread count; oracle/rbref.cpp "
                          f"RoaringBitmap.{['and', 'or', 'xor', 'andNot'][op]} (C++ restatement, -O3), pairs split "
                          "over the threads")


# ------------------------------------------------------------------------------- config 1
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


def run_census(args, ctx, rb, steps=50, warmup=5):
    """Config 1: RealDataBenchmark{And,Or,Xor,AndNot} on census1881 — 199 consecutive pairs (k, k+1)
    of the 200 bitmaps (bitmapOf), one batched call per op; a step is the four ops."""
    vals = load_census()
    s = ctx.upload_values(vals)
    n = len(vals) - 1
    ai = np.arange(n, dtype=np.uint32)
    bi = ai + 1
    ops = {k: getattr(rb, k) for k in OPS}
    cards = {k: int(ctx.pairwise(op, s, s, ai, bi).cardinalities().sum()) for k, op in ops.items()}
    # algorithmic bytes of one sweep (deterministic per op), and the device-side call breakdown
    step_bytes, step_ops, calls = 0, 0, {}
    os.environ["RBGPU_SMALL_KERNEL_TIMES"] = "1"  # per-kernel events for this breakdown only
    for k, op in ops.items():
        lib_us = []
        for _ in range(20):
            ctx.pairwise(op, s, s, ai, bi).close()
            st = ctx.stats()
            lib_us.append(st["call_us"])
        step_bytes += st["input_bytes"]
        step_ops += st["tasks"]
        calls[k] = {"device_ms": round(st["total_ms"], 4), "c_call_us_median": round(float(np.median(lib_us)), 1),
                    "kernels": {x["name"]: round(x["ms"], 4) for x in st["kernels"]}}
    del os.environ["RBGPU_SMALL_KERNEL_TIMES"]
    for k, op in ops.items():  # the C call's own wall time without the breakdown's events
        lib_us = []
        for _ in range(20):
            ctx.pairwise(op, s, s, ai, bi).close()
            lib_us.append(ctx.stats()["call_us"])
        calls[k]["c_call_us_median"] = round(float(np.median(lib_us)), 1)
    for _ in range(warmup):
        for op in ops.values():
            ctx.pairwise(op, s, s, ai, bi).close()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        for op in ops.values():
            ctx.pairwise(op, s, s, ai, bi).close()
    ctx.synchronize()
    el = time.perf_counter() - t0
    in_bytes = step_bytes * steps
    out = {"workload": "config1: census1881 RealDataBenchmark and/or/xor/andNot, 199 consecutive pairs per op",
           "value": round(in_bytes / el / 1e9, 3), "unit": "GB/s", "steps": steps,
           "ms_per_step": round(el / steps * 1e3, 4),
           "us_per_op_sweep": round(el / steps / 4 * 1e6, 1), "cardinality_sums": cards,
           "container_ops_per_s": round(step_ops * steps / el, 1),
           "container_ops_unit": "matched container pairs + copied unmatched containers of the 4 x 199 pairs",
           "golden_ok": cards == CENSUS_EXPECTED, "calls": calls,
           "note": "us_per_op_sweep = wall time of one batched call (199 pairs, one op) through the Python "
                   "binding, results materialized in HBM; device_ms = the call's span on the GPU stream"}
    if not args.no_cpu_baseline:
        from oracle import rbref as R
        refs = [R.RefBitmap.deserialize(x) for x in s.serialize()]
        a_r, b_r = refs[:-1], refs[1:]

        def sweep(th):
            for op in ops.values():
                R.pairwise_batch(op, a_r, b_r, threads=th)
        rates = multi_rate(sweep, 3.0)
        out["cpu_baseline"] = baseline_entry(in_bytes / steps, rates, "port",
                                             "the whole config (199 pairs x 4 ops), oracle/rbref.cpp",
                                             {"us_per_op_sweep_1thread": round(1e6 / rates[1] / 4, 1),
                                              "us_per_op_sweep_best": round(1e6 / max(rates.values()) / 4, 1)})
    s.close()
    return out


# ------------------------------------------------------------------------------- config 5
BSI_NSLICES, BSI_NROWS = 64, 100_000_000
BSI_LO, BSI_HI = 0x3A00_0000_0000_0000, 0xB100_0000_0000_0000  # a mid-range window: no min/max shortcut


def run_bsi(args, D, ctx, rb, steps=5, warmup=2):
    """Config 5: Roaring64BitmapSliceIndex.compare(RANGE, lo, hi, null) over 64 slices x 100M rows
    (runOptimize'd BSI, random value bits) — one fused pass per high key for both O'Neil chains.
    At N > 1 rank r holds and answers its high-key range (ShardedBsi; strong scaling)."""
    from roaringbitmap_amd.sharding import ShardedBsi
    nkeys = (BSI_NROWS + 65535) // 65536
    lo_k, hi_k = (nkeys * D.rank) // D.world, (nkeys * (D.rank + 1)) // D.world
    if D.rank == D.world - 1:
        hi_k = 65536
    kr = (lo_k, hi_k)
    d = ctx.generate_bsi(BSI_NSLICES, BSI_NROWS, seed=42, key_range=kr if D.world > 1 else None)
    vmin, vmax = 0, (1 << BSI_NSLICES) - 1
    comm = D.comm
    sb = ShardedBsi(D.td, D.rank, D.world, D.device) if D.td is not None and comm is None else None

    def step():
        if comm is not None:  # rbgpu_bsi_compare_sharded: local key range + summary all-gather in librbgpu
            r, summ = comm.bsi_compare_sharded(rb.BSI_RANGE, d, BSI_LO, BSI_HI, vmin, vmax, kr)
            st, card = ctx.stats_raw(), summ["cardinality"]
        else:
            r = ctx.bsi_compare(rb.BSI_RANGE, d, BSI_LO, BSI_HI, vmin, vmax, key_range=kr)
            st = ctx.stats_raw()  # the struct; converted to a dict after the timed loop
            card = sb.finish(r, kr, r.summaries()[0]).cardinality if sb is not None else None
        r.close()
        return st, card

    from roaringbitmap_amd.engine import stats_dict
    el, sts = timed(D, ctx, steps, warmup, step)
    sts = [(stats_dict(s), c) for s, c in sts]
    in_b = sum(s["input_bytes"] for s, _ in sts)
    tot_in = D.reduce([float(in_b)])[0]
    last = sts[-1][0]
    km = float(np.mean([s["main_kernel_ms"] for s, _ in sts]))
    kb = float(np.mean([s["main_kernel_bytes"] for s, _ in sts]))
    card = sts[-1][1] if sb is not None else int(last["result_cardinality"])
    ts = d.type_stats()
    # O'Neil chain steps: per active high key, one per slice and comparator (GE, LE) and the final AND
    chain_keys = float(np.mean([s["kernels"][0]["items"] for s, _ in sts])) / 2 if last["kernels"] else 0.0
    tot_ops = D.reduce([chain_keys * (2 * BSI_NSLICES + 1) * steps])[0]
    out = {"workload": f"config5: BSI compare RANGE over {BSI_NSLICES} slices x {BSI_NROWS} rows (2 O'Neil chains "
                       "+ AND, fused into one pass per key)",
           "value": round(tot_in / el / 1e9, 3), "unit": "GB/s", "n_gpus": D.world, "steps": steps,
           "ms_per_step": round(el / steps * 1e3, 4), "step_ms": step_spread(D), "scaling": "strong",
           "result_cardinality": card, "containers_rank0": ts,
           "container_ops_per_s": round(tot_ops / el, 1),
           "container_ops_unit": f"container ops of the chains, all ranks: per high key {BSI_NSLICES} slices x 2 "
                                 "comparators (GE, LE) + the final AND",
           "parallelism": (f"high-key range shards x{D.world}, per step all_gather of shard summaries over "
                           + ("librbgpu's RCCL communicator (rbgpu_bsi_compare_sharded)" if comm is not None
                              else "torch.distributed (ShardedBsi)")) if D.world > 1 else "single GPU",
           "key_range_rank0": list(kr),
           "roofline": roofline(last["main_kernel"], km, kb, pmc_traffic("rbg::k_bsi_range"), D, {
               "note": "the fused kernel reads every slice container once for both comparators (GE and LE); "
                       "algorithmic bytes count that one read"})}
    # the index's key tables, built on its first compare (the warmup) and kept with the set: what a caller
    # that builds a fresh index per query pays on top of the step
    su = d.setup_parts()["bsi_tables"]
    out["setup"] = {"ms": su["ms"], "bytes": su["bytes"],
                    "what": "rbgpu_set_setup_parts[3] of this rank's index: key -> container tables of its slices "
                            "and ebM, and ebM's key list, once per index before the warmup step, not inside the "
                            "timed steps"}
    with_setup = el / steps * 1e3 + D.reduce([float(su["ms"])], "max")[0]
    out["ms_per_step_with_setup"] = round(with_setup, 4)
    out["value_with_setup"] = round(tot_in / steps / (with_setup * 1e-3) / 1e9, 3)
    d.close()
    if not args.no_cpu_baseline and D.world == 1:
        out["cpu_baseline"] = bsi_cpu_baseline(ctx, rb)
    return out


def bsi_cpu_baseline(ctx, rb, seconds=4.0):
    """The oracle's compare on the first high keys of the same index (2 per host CPU, at least 64): the C++
    O'Neil chain over rbref.cpp's static ops (rbref_bsi_compare_keys, pinned to the Python restatement by
    test_bsi_cpp_twin_matches_restatement), 1 thread, then key-parallel over the host CPUs in contiguous key
    ranges (the split BitSliceIndexBase.java:99-166 uses).  No interpreter in the loop, so the thread counts
    measure the algorithm (the Python composition measured the GIL)."""
    from oracle import rbref as R
    nkeys = min(max(64, 2 * ALL_CORES), (BSI_NROWS + 65535) // 65536)
    vmin, vmax = 0, (1 << BSI_NSLICES) - 1
    per_key = []
    for k in range(nkeys):
        s = ctx.generate_bsi(BSI_NSLICES, BSI_NROWS, seed=42, key_range=(k, k + 1))
        refs = [R.RefBitmap.deserialize(x) for x in s.serialize()]
        s.close()
        per_key.append((refs[:-1], refs[-1]))
    s = ctx.generate_bsi(BSI_NSLICES, BSI_NROWS, seed=42, key_range=(0, nkeys))
    r = ctx.bsi_compare(rb.BSI_RANGE, s, BSI_LO, BSI_HI, vmin, vmax)
    st = ctx.stats()
    sb, want_card = st["input_bytes"], st["result_cardinality"]
    r.close()
    s.close()
    got = R.bsi_compare_keys(per_key, R.BSI_RANGE, BSI_LO, BSI_HI, vmin, vmax, 1)
    assert got == want_card, (got, want_card)  # the baseline computes the device's answer
    rates = multi_rate(lambda th: R.bsi_compare_keys(per_key, R.BSI_RANGE, BSI_LO, BSI_HI, vmin, vmax, th), seconds)
    return baseline_entry(sb, rates, "port",
                          f"the same query on the first {nkeys} high keys ({nkeys} x 65536 rows, {sb} algorithmic "
                          "input bytes); oracle/rbref.cpp rbref_bsi_compare_keys (C++ O'Neil chains over the static "
                          "ops, keys split over the threads)")


# ------------------------------------------------------------------------------- configs 3 / 4
WIDE_WORKLOADS = {
    # name: (generator workload, semantics, default bitmaps, PMC kernel, CPU sample keys, description)
    "wide_or": ("WL_WIDE_DENSE", "FAST_OR", 1024, "rbg::k_wide_reduce<0>", 1024,
                "config3: FastAggregation.or of {n} dense bitmaps over the full 2^32 universe"),
    "wide_and_runs": ("WL_WIDE_RUNS", "FAST_AND", 4096, "rbg::k_wide_runs_and", 256,
                      "config4: FastAggregation.and (workShyAnd) of {n} run-heavy bitmaps x 65536 keys"),
    "wide_xor_runs": ("WL_WIDE_RUNS", "FAST_XOR", 4096, "rbg::k_wide_runs_xor", 256,
                      "config4: FastAggregation.xor (naive_xor) of {n} run-heavy bitmaps x 65536 keys"),
}
# the all-core CPU baseline of each wide semantic: ParallelAggregation where the reference has one,
# else the same per-key semantic key-parallel (oracle rbref_wide_mt)
WIDE_PARALLEL = {"FAST_OR": "PAR_OR", "FAST_XOR": "PAR_XOR", "FAST_AND": "FAST_AND"}
# the derived per-set items (rbgpu_set_setup_parts) each wide path builds on a fresh set (workShyAnd reads the
# set's own run counts and offsets since round 6: no packed records)
WIDE_SETUP_PARTS = {"FAST_OR": ("dense_check",), "FAST_AND": ("dense_check",),
                    "FAST_XOR": ("dense_check", "krec")}
# bytes per container a config-4 kernel must read besides the payload arena (at least once per launch):
# naive_xor its key-major 4-B record, workShyAnd the u16 run count and the u64 payload offset
WIDE_META_BYTES = {"FAST_XOR": 4, "FAST_AND": 10}


def run_wide(args, name, D, ctx, rb, nbitmaps, steps, warmup, a=None):
    """Key-range-sharded wide aggregation: rank r generates and aggregates keys [lo_r, hi_r) of the
    one global dataset (strong scaling: total work fixed), then the RCCL exchange of the shard
    summaries (roaringbitmap_amd.sharding).  The synthetic data is uniform over keys, so equal key
    ranges are byte-balanced; partition_keys() does the same from rbgpu_set_key_bytes for real data."""
    from roaringbitmap_amd.sharding import ShardedWide
    wl, sem_name, _, pmc_name, _, desc = WIDE_WORKLOADS[name]
    lo, hi = (65536 * D.rank) // D.world, (65536 * (D.rank + 1)) // D.world
    own = a is None
    if own:
        a = ctx.generate_keys(getattr(rb, wl), nbitmaps, lo, hi, seed=42)
    from roaringbitmap_amd.sharding import ShardResult
    sem = getattr(rb, sem_name)
    comm = D.comm
    sw = ShardedWide(D.td, D.rank, D.world, device=D.device) if D.td is not None and comm is None else None

    def step():
        if comm is not None:  # rbgpu_wide_sharded: local key range + summary all-gather in librbgpu
            r, summ = comm.wide_sharded(sem, a, (lo, hi))
            st = ctx.stats()
            res = ShardResult(r, (lo, hi), summ["cardinality"], summ["n_containers"], summ["n_run_containers"],
                              summ["payload_bytes"], summ["serialized_size"], summ["payload_offset"])
        elif sw is None:
            r = ctx.wide(sem, a, key_range=(lo, hi))
            st, res = ctx.stats(), None
        else:
            res = sw.aggregate(ctx, sem, a, (lo, hi))
            r = res.local
            st = ctx.stats()
        r.close()
        return st, res

    el, sts = timed(D, ctx, steps, warmup, step)
    in_b = sum(s["input_bytes"] for s, _ in sts)
    ts = a.type_stats()
    local_conts = sum(int(ts[k]) for k in ("array", "bitmap", "run"))
    total_in, total_ops = D.reduce([float(in_b), float(local_conts * steps)])
    last, res = sts[-1]
    k_ms = float(np.mean([s["main_kernel_ms"] for s, _ in sts]))
    k_bytes = float(np.mean([s["main_kernel_bytes"] for s, _ in sts]))
    out = {
        "workload": desc.format(n=nbitmaps),
        "value": round(total_in / el / 1e9, 3), "unit": "GB/s", "n_gpus": D.world, "steps": steps,
        "ms_per_step": round(el / steps * 1e3, 4), "step_ms": step_spread(D), "scaling": "strong",
        "input_bytes_per_step": int(total_in // steps),
        "container_ops_per_s": round(total_ops / el, 1),
        "container_ops_unit": "input containers folded per step, all ranks (each member container enters "
                              "its key's reduction once)",
        "key_range_rank0": [lo, hi],
        "containers_rank0": ts,
        "parallelism": (f"key-range shards x{D.world}; per step all_gather of shard summaries (cardinality, "
                        "containers, Run containers, payload bytes) over "
                        + ("librbgpu's RCCL communicator (rbgpu_wide_sharded)" if comm is not None
                           else "torch.distributed (ShardedWide)")) if D.world > 1 else "single GPU",
        "roofline": roofline(last["main_kernel"], k_ms, k_bytes, pmc_traffic(pmc_name), D),
    }
    if sem_name in WIDE_META_BYTES:
        # the traffic calibration's known byte count: every metadata record and every payload
        # byte of the set must come from HBM at least once per launch (the arena is GBs, far past the 256 MiB
        # Infinity Cache), plus the results written; the PMC figure is checked against it
        prov = WIDE_META_BYTES[sem_name] * local_conts + a.payload_capacity
        rl = out["roofline"]
        rl["provable_min_read_bytes"] = int(prov)
        if rl.get("traffic"):
            rl["traffic_vs_provable_read"] = round(rl["traffic"] / prov, 3)
    # the per-set metadata the kernels derived on the set's first use (outside the timed steps; a caller
    # that uploads a fresh set per call pays it once per set): the items this line's path needs on a fresh set
    parts = a.setup_parts()
    need = WIDE_SETUP_PARTS[sem_name]
    su = {"ms": round(sum(parts[k]["ms"] for k in need), 4), "bytes": sum(parts[k]["bytes"] for k in need)}
    out["setup"] = {"ms": su["ms"], "bytes": su["bytes"], "parts": {k: parts[k] for k in need},
                    "what": "rbgpu_set_setup_parts of this rank's set: the derived metadata this path builds on a "
                            "fresh set (dense-layout check; naive_xor: key-major 4-B records straight from the set's "
                            "metadata, k_records_direct2; workShyAnd reads the set's own metadata and builds none), "
                            "once per set before the warmup step, not inside the timed steps"}
    # what a caller that uploads a fresh set for every call pays (the reference builds its per-call state each
    # time: FastAggregation.java:356-396, 576-582): the step plus this path's setup, max over ranks
    su_ms = D.reduce([float(su["ms"])], "max")[0]
    with_setup = el / steps * 1e3 + su_ms
    out["ms_per_step_with_setup"] = round(with_setup, 4)
    out["value_with_setup"] = round(total_in / steps / (with_setup * 1e-3) / 1e9, 3)
    out["roofline_pct_with_setup"] = round(100.0 * out["value_with_setup"] / (HBM_PEAK_GBS * D.world), 2)
    out["result_cardinality"] = res.cardinality if res is not None else int(last["result_cardinality"])
    if res is not None:
        out["result_serialized_bytes"] = res.serialized_size
    if own:
        a.close()
    return out


def wide_cpu_baseline(ctx, rb, name, seconds: float):
    """The oracle's FastAggregation (C++ restatement) on the first K high keys of the same dataset:
    1 thread with the FastAggregation semantic, then all host CPUs with ParallelAggregation's
    key-parallel restatement (ParallelAggregation.java:161-223; rbref_wide_mt)."""
    from oracle import rbref as R
    wl, sem_name, n, _, nkeys, _ = WIDE_WORKLOADS[name]
    a = ctx.generate_keys(getattr(rb, wl), n, 0, nkeys, seed=42)
    refs = [R.RefBitmap.deserialize(x) for x in a.serialize()]
    r = ctx.wide(getattr(rb, sem_name), a)
    sample_bytes = ctx.stats()["input_bytes"]
    r.close()
    a.close()
    sem, par = getattr(R, sem_name), getattr(R, WIDE_PARALLEL[sem_name])
    rates = multi_rate(lambda th: R.wide(sem, refs) if th == 1 else R.wide_mt(par, refs, th), seconds)
    return baseline_entry(sample_bytes, rates, "port",
                          f"keys [0, {nkeys}) of the {n} generated bitmaps ({sample_bytes} algorithmic input bytes); "
                          f"1 thread: oracle/rbref.cpp {sem_name}; more threads: {WIDE_PARALLEL[sem_name]} "
                          f"key-parallel restatement (rbref_wide_mt); ~{seconds / len(rates):.1f}s each")


# ------------------------------------------------------------------------------- main
def main():
    args = parse()
    D = Dist()
    import roaringbitmap_amd as rb
    ctx = rb.Context(D.local)
    D.open_comm(ctx)
    seed = 42 + D.rank
    sec = SECONDARY_ALL if args.secondary == "all" else \
        ([] if args.secondary == "none" else [s for s in args.secondary.split(",") if s])
    line = {"metric": METRIC, "higher_is_better": True, "vs_baseline": None, "dtype": "u64",
            "n_gpus": D.world, "steps": args.steps, "warmup": args.warmup,
            "data": "synthetic (device SplitMix64 generator, runOptimize'd containers; SURVEY §8d)"}
    if D.comm_error:
        line["comm_fallback"] = D.comm_error
    secondary = {}

    if args.workload in WIDE_WORKLOADS or args.workload == "bsi_range":
        if args.workload == "bsi_range":
            w = run_bsi(args, D, ctx, rb, args.steps, args.warmup)
        else:
            nb = args.wide_bitmaps or WIDE_WORKLOADS[args.workload][2]
            w = run_wide(args, args.workload, D, ctx, rb, nb, args.steps, args.warmup)
            if D.world == 1 and not args.no_cpu_baseline:
                w["cpu_baseline"] = wide_cpu_baseline(ctx, rb, args.workload, args.cpu_seconds / 2)
        line.update({"value": w["value"], "unit": "GB/s", "ms_per_step": w["ms_per_step"], "step_ms": w["step_ms"],
                     "scaling": "strong",
                     "config": {k: v for k, v in w.items() if k not in ("value", "roofline", "ms_per_step", "step_ms",
                                                                        "cpu_baseline", "unit", "steps", "n_gpus")},
                     "roofline": w["roofline"]})
        if "cpu_baseline" in w:
            line["cpu_baseline"] = w["cpu_baseline"]
        if D.rank == 0:
            print(json.dumps(line), flush=True)
        D.close()
        return

    op = {"pairwise_and": rb.AND, "pairwise_or": rb.OR, "pairwise_xor": rb.XOR, "pairwise_andnot": rb.ANDNOT}[
        args.workload]
    a, b = ctx.generate(rb.WL_FILTER_POSTING, args.pairs, seed=seed)
    ctx.synchronize()
    h = pairwise_line(D, ctx, rb, a, b, op, args.steps, args.warmup, args.pairs)
    line.update({"value": h["value"], "unit": "GB/s", "ms_per_step": h["ms_per_step"], "step_ms": h["step_ms"],
                 "scaling": "weak",
                 "config": {"workload": h["workload"], "units_per_gpu": args.pairs, "unit": "pairs",
                            "input_bytes_per_step_per_gpu": h["input_bytes_per_step_per_gpu"],
                            "output_bytes_per_step_per_gpu": h["output_bytes_per_step_per_gpu"],
                            "roofline_pct_whole_step": h["roofline_pct_whole_step"],
                            "container_ops_per_s": h["container_ops_per_s"],
                            "container_ops_unit": h["container_ops_unit"],
                            "result_cardinality_all_ranks": h["result_cardinality_all_ranks"],
                            "containers_a_rank0": a.type_stats(), "containers_b_rank0": b.type_stats(),
                            "parallelism": h["parallelism"]},
                 "roofline": h["roofline"]})
    if D.world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = pairwise_cpu_baseline(ctx, a, b, op, args.cpu_seconds)
    if "pairwise_async" in sec:
        secondary["pairwise_" + OPS[op].lower() + "_async"] = pairwise_async_line(
            D, ctx, rb, a, b, op, args.steps, args.warmup, h["input_bytes_per_step_per_gpu"],
            h["output_bytes_per_step_per_gpu"], None)
    if "pairwise_ops" in sec:
        for o in range(4):
            if o == op:
                continue
            w = pairwise_line(D, ctx, rb, a, b, o, max(3, args.steps // 2), 1, args.pairs)
            if D.world == 1 and not args.no_cpu_baseline:
                w["cpu_baseline"] = pairwise_cpu_baseline(ctx, a, b, o, 4.0, sample=20000)
            secondary["pairwise_" + OPS[o].lower()] = w
    a.close()
    b.close()
    if "census" in sec and D.world == 1:
        secondary["census1881"] = run_census(args, ctx, rb)
    if "bsi_range" in sec:
        secondary["bsi_range"] = run_bsi(args, D, ctx, rb)
    def wide_secondary(name, data=None):
        w = run_wide(args, name, D, ctx, rb, WIDE_WORKLOADS[name][2], 3, 1, a=data)
        if D.world == 1 and not args.no_cpu_baseline:
            w["cpu_baseline"] = wide_cpu_baseline(ctx, rb, name, 4.0)
        secondary[name] = w

    if "wide_or" in sec:
        wide_secondary("wide_or")
    # naive_xor first: on the fresh set it builds its key-major records from the metadata (k_records_direct),
    # as a caller's first naive_xor would; workShyAnd then adds its packed records
    c4 = [n for n in ("wide_xor_runs", "wide_and_runs") if n in sec]
    if c4:  # config 4 AND and XOR read the same dataset: generate this rank's key range once
        lo, hi = (65536 * D.rank) // D.world, (65536 * (D.rank + 1)) // D.world
        data = ctx.generate_keys(rb.WL_WIDE_RUNS, WIDE_WORKLOADS["wide_and_runs"][2], lo, hi, seed=42)
        for name in c4:
            wide_secondary(name, data)
        data.close()
    if D.rank == 0:
        for name, w in secondary.items():  # one line per secondary workload, before the headline
            print(json.dumps({"secondary_line": name, **w}), flush=True)
    if secondary:
        line["secondary"] = secondary
        # the headline line ends with a compact summary, so a tail of the output holds every workload
        line["secondary_summary"] = {n: secondary_summary(w) for n, w in secondary.items()}
    if D.rank == 0:
        print(json.dumps(line), flush=True)
    D.close()


def secondary_summary(w: dict) -> dict:
    rl = w.get("roofline", {})
    out = {"ms": w.get("ms_per_step"), "GB/s": w.get("value"), "frac": rl.get("frac"),
           "whole_pct": w.get("roofline_pct_whole_step"), "cops": w.get("container_ops_per_s")}
    if "setup" in w:
        out["setup_ms"] = w["setup"]["ms"]
        out["ms_with_setup"] = w.get("ms_per_step_with_setup")
        out["GB/s_with_setup"] = w.get("value_with_setup")
    cb = w.get("cpu_baseline")
    if cb:
        out["cpu"] = cb.get("value")
    return {k: v for k, v in out.items() if v is not None}


if __name__ == "__main__":
    main()
