"""Device RoaringFormatSpec codec throughput (codec.hip) on a config-2 sized set: serialize into HBM,
parse it back from HBM, check the round trip on the device.  Bytes/s counts the serialized bytes.
Also times the host codec (RBGPU_HOST_CODEC=1: download + format.cpp / format.cpp + upload) for scale.
usage: python scripts/codec_bench.py [--bitmaps N] [--reps R]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import roaringbitmap_amd as rb  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bitmaps", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--host-sample", type=int, default=1 << 16)
    args = ap.parse_args()
    torch.cuda.init()
    ctx = rb.Context(0)
    a, _ = ctx.generate(rb.WL_FILTER_POSTING, args.bitmaps, seed=42)
    total = int(a.serialized_sizes().sum())
    buf = torch.empty(total + 64, dtype=torch.uint8, device="cuda:0")
    buf2 = torch.empty_like(buf)
    torch.cuda.synchronize()
    res = {"bitmaps": args.bitmaps, "containers": a.n_containers, "serialized_bytes": total}
    t = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        offs = a.serialize_device(buf.data_ptr(), buf.numel())
        t.append(time.perf_counter() - t0)
    res["serialize_ms"] = 1e3 * min(t)
    t = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        b = ctx.upload_serialized_device(buf.data_ptr(), offs)
        t.append(time.perf_counter() - t0)
        last = b
    res["deserialize_ms"] = 1e3 * min(t)
    last.serialize_device(buf2.data_ptr(), buf2.numel())
    torch.cuda.synchronize()
    res["round_trip_equal"] = bool(torch.equal(buf[:total], buf2[:total]))
    res["serialize_GBps"] = total / res["serialize_ms"] / 1e6
    res["deserialize_GBps"] = total / res["deserialize_ms"] / 1e6
    # host codec on a sample, for scale
    n = min(args.host_sample, args.bitmaps)
    t0 = time.perf_counter()
    blobs = a.serialize(0, n)
    t_dev_host = time.perf_counter() - t0
    os.environ["RBGPU_HOST_CODEC"] = "1"
    t0 = time.perf_counter()
    blobs_h = a.serialize(0, n)
    t_host_ser = time.perf_counter() - t0
    t0 = time.perf_counter()
    ctx.upload_serialized(blobs_h)
    t_host_de = time.perf_counter() - t0
    os.environ.pop("RBGPU_HOST_CODEC")
    t0 = time.perf_counter()
    ctx.upload_serialized(blobs_h)
    t_dev_de = time.perf_counter() - t0
    sb = sum(len(x) for x in blobs)
    res["sample_bitmaps"] = n
    res["sample_equal"] = blobs == blobs_h
    res["host_buffers_GBps"] = {"serialize_device_codec": sb / t_dev_host / 1e9, "serialize_host_codec": sb / t_host_ser / 1e9,
                                "deserialize_device_codec": sb / t_dev_de / 1e9, "deserialize_host_codec": sb / t_host_de / 1e9}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
