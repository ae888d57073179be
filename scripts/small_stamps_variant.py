"""Study build: k_pair_small with per-block s_memrealtime stamps (RBGPU_SMALL_STAMPS=1 prints a timeline
to stderr), as abvar/<name>/librbgpu.so.  The product sources are patched only for the build and restored.

usage: python scripts/small_stamps_variant.py NAME [DEF=1 ...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from roaringbitmap_amd import build as b  # noqa: E402

CS = os.path.join(ROOT, "roaringbitmap_amd", "csrc")
P = {f: os.path.join(CS, f) for f in ("kernels.hpp", "pairwise.hip", "api.hip")}


def sub(text, old, new):
    assert old in text, old[:80]
    return text.replace(old, new, 1)


def patched(src):
    k, p, a = src["kernels.hpp"], src["pairwise.hip"], src["api.hip"]
    k = sub(k, "  OutView out;\n};", "  OutView out;\n  uint64_t *stamps;\n};")
    k = sub(k, "static_assert(sizeof(SmallTabInline) + sizeof(SmallPairArgs) + 16 <= 4096", "static_assert(true || 1")
    p = sub(p, "  const int lane = lane_id(), wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);\n  // the block's pair",
            "  const int lane = lane_id(), wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);\n"
            "  const uint64_t st0 = __builtin_amdgcn_s_memrealtime();\n  // the block's pair")
    p = sub(p, "  // ---- one wave per merged key\n", "  const uint64_t st1 = __builtin_amdgcn_s_memrealtime();\n  // ---- one wave per merged key\n")
    p = sub(p, "  // slots past the merged keys hold nothing\n",
            "  __syncthreads();\n  const uint64_t st2 = __builtin_amdgcn_s_memrealtime();\n  // slots past the merged keys hold nothing\n")
    p = sub(p, "  __syncthreads();\n  if (!s_last) return;\n  small_compact(a, tab, reinterpret_cast<uint32_t *>(dyn_lds), wtot);\n",
            "  __syncthreads();\n"
            "  if (threadIdx.x == 0) { a.stamps[5ull * blockIdx.x] = st0; a.stamps[5ull * blockIdx.x + 1] = st1;\n"
            "    a.stamps[5ull * blockIdx.x + 2] = st2; a.stamps[5ull * blockIdx.x + 3] = __builtin_amdgcn_s_memrealtime(); }\n"
            "  if (!s_last) return;\n  small_compact(a, tab, reinterpret_cast<uint32_t *>(dyn_lds), wtot);\n"
            "  __syncthreads();\n"
            "  if (threadIdx.x == 0) a.stamps[5ull * blockIdx.x + 4] = __builtin_amdgcn_s_memrealtime();\n")
    a = sub(a, "  sa.ctr = ctx->d_small_ctr;\n",
            "  sa.ctr = ctx->d_small_ctr;\n  std::vector<uint64_t> hst;\n"
            "  { uint64_t *d = nullptr; if (hipMalloc((void **)&d, 40ull * nblocks) != hipSuccess) return 1;\n"
            "    (void)hipMemset(d, 0, 40ull * nblocks); sa.stamps = d; hst.resize(5ull * nblocks); }\n")
    a = sub(a, "  const uint64_t nres = hout[0];\n  const KernelSpan spans[1]",
            "  const uint64_t nres = hout[0];\n"
            "  if (getenv(\"RBGPU_SMALL_STAMPS\")) {\n"
            "    (void)hipMemcpy(hst.data(), sa.stamps, 40ull * nblocks, hipMemcpyDeviceToHost);\n"
            "    uint64_t t0 = ~0ull, tw = 0, tc = 0, tcs = 0; uint32_t il = 0;\n"
            "    std::vector<double> al, wk, fin;\n"
            "    for (uint32_t i = 0; i < nblocks; ++i) { const uint64_t *h = &hst[5ull * i]; t0 = std::min(t0, h[0]);\n"
            "      if (h[2] > tw) { tw = h[2]; il = i; } if (h[4]) { tc = h[4]; tcs = h[3]; }\n"
            "      al.push_back((h[1] - h[0]) / 100.0); wk.push_back((h[2] - h[1]) / 100.0); fin.push_back((h[3] - h[2]) / 100.0); }\n"
            "    uint64_t late = 0; for (uint32_t i = 0; i < nblocks; ++i) late = std::max(late, hst[5ull * i] - t0);\n"
            "    auto pct = [](std::vector<double> v, double q) { std::sort(v.begin(), v.end()); return v[(size_t)(q * (v.size() - 1))]; };\n"
            "    uint32_t pl = 0; for (uint32_t p = 0; p < np; ++p) if ((inl ? (uint32_t)ti->blk[p] : blk[p]) <= il) pl = p;\n"
            "    const uint64_t *h = &hst[5ull * il];\n"
            "    fprintf(stderr, \"stamps blocks %u E %llu kpw %u | last start +%.2f | align p50 %.2f max %.2f | work p50 %.2f p90 %.2f max %.2f | \"\n"
            "      \"counters p50 %.2f max %.2f | latest work end +%.2f (block %u pair %u nk %u: start +%.2f align %.2f work %.2f) | \"\n"
            "      \"last add +%.2f compaction end +%.2f\\n\", nblocks, (unsigned long long)E, kpw, late / 100.0, pct(al, .5), pct(al, 1),\n"
            "      pct(wk, .5), pct(wk, .9), pct(wk, 1), pct(fin, .5), pct(fin, 1), (tw - t0) / 100.0, il, pl,\n"
            "      (unsigned)(slot[pl + 1] - slot[pl]), (h[0] - t0) / 100.0, (h[1] - h[0]) / 100.0, (h[2] - h[1]) / 100.0,\n"
            "      (tcs - t0) / 100.0, (tc - t0) / 100.0);\n"
            "  }\n  (void)hipFree(sa.stamps);\n"
            "  const KernelSpan spans[1]")
    a = sub(a, "#include", "#include <algorithm>\n#include <vector>\n#include")
    return {"kernels.hpp": k, "pairwise.hip": p, "api.hip": a}


def main():
    name, defs = sys.argv[1], sys.argv[2:]
    orig = {f: open(P[f]).read() for f in P}
    try:
        for f, t in patched(orig).items():
            open(P[f], "w").write(t)
        os.makedirs(os.path.join(ROOT, "abvar", name), exist_ok=True)
        print(b.build(defines=defs, out=os.path.join(ROOT, "abvar", name, "librbgpu.so"),
                      obj=os.path.join(ROOT, "scratch", name, "obj")))
    finally:
        for f, t in orig.items():
            open(P[f], "w").write(t)


if __name__ == "__main__":
    main()
