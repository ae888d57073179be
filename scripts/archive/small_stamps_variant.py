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
    p = sub(p, "    p = lo;\n  }\n", "    p = lo;\n  }\n  const uint64_t stA = __builtin_amdgcn_s_memrealtime();\n")
    p = sub(p, "  for (uint32_t t = threadIdx.x; t < nb; t += nt) K[na + t] = a.B.key[j0 + t];\n  __syncthreads();\n",
            "  for (uint32_t t = threadIdx.x; t < nb; t += nt) K[na + t] = a.B.key[j0 + t];\n  __syncthreads();\n"
            "  const uint64_t stB = __builtin_amdgcn_s_memrealtime();\n")
    p = sub(p, "  // ---- one wave per merged key\n", "  const uint64_t st1 = __builtin_amdgcn_s_memrealtime();\n  // ---- one wave per merged key\n")
    p = sub(p, "  for (uint32_t k = 0; k * W < nu; ++k) {\n",
            "  uint64_t wt[4] = {__builtin_amdgcn_s_memrealtime(), 0, 0, 0}, ms[3] = {0, 0, 0};\n  uint32_t wflags = 0, wk = 0;\n"
            "  for (uint32_t k = 0; k * W < nu; ++k) {\n")
    p = sub(p, "        if (!CARD_ONLY) outb += alg_bytes(ty, (uint32_t)c, (uint32_t)nr) + 16;\n      }\n    }\n  }\n",
            "        if (!CARD_ONLY) outb += alg_bytes(ty, (uint32_t)c, (uint32_t)nr) + 16;\n      }\n    }\n"
            "    if (wk < 3) { wt[1 + wk] = __builtin_amdgcn_s_memrealtime(); wflags |= (has_a && has_b ? 1u : 0u) << wk; }\n"
            "    ++wk;\n  }\n"
            "  if (lane == 0) { uint64_t *q = a.stamps + 8ull * a.nblocks + 8ull * (4ull * blockIdx.x + wv);\n"
            "    q[0] = wt[0]; q[1] = wt[1]; q[2] = wt[2]; q[3] = wt[3]; q[4] = wflags | (wk << 8); q[5] = ms[0]; q[6] = ms[1]; q[7] = ms[2]; }\n")
    p = sub(p, "      if (lane == 0) inb += alg_bytes(kArray, ca, 0) + alg_bytes(kArray, cb, 0) + 32;\n",
            "      if (lane == 0) inb += alg_bytes(kArray, ca, 0) + alg_bytes(kArray, cb, 0) + 32;\n"
            "      __builtin_amdgcn_s_waitcnt(0); if (!ms[0]) ms[0] = __builtin_amdgcn_s_memrealtime();\n")
    p = sub(p, "        merge_stage(q, ca, r, cb, s, lane);\n      }\n",
            "        merge_stage(q, ca, r, cb, s, lane);\n      }\n      if (!ms[1]) ms[1] = __builtin_amdgcn_s_memrealtime();\n")
    p = sub(p, "      c = (int)merge_run<OP, !CARD_ONLY>(s, ca, cb, reinterpret_cast<uint16_t *>(dst), lane);\n",
            "      c = (int)merge_run<OP, !CARD_ONLY>(s, ca, cb, reinterpret_cast<uint16_t *>(dst), lane);\n"
            "      __builtin_amdgcn_s_waitcnt(0); if (!ms[2]) ms[2] = __builtin_amdgcn_s_memrealtime();\n")
    p = sub(p, "  // slots past the merged keys hold nothing\n",
            "  __syncthreads();\n  const uint64_t st2 = __builtin_amdgcn_s_memrealtime();\n  // slots past the merged keys hold nothing\n")
    p = sub(p, "  __syncthreads();\n  if (!s_last) return;\n  small_compact(a, tab, reinterpret_cast<uint32_t *>(dyn_lds), wtot);\n",
            "  __syncthreads();\n"
            "  if (threadIdx.x == 0) { a.stamps[8ull * blockIdx.x] = st0; a.stamps[8ull * blockIdx.x + 1] = st1;\n"
            "    a.stamps[8ull * blockIdx.x + 5] = stA; a.stamps[8ull * blockIdx.x + 6] = stB;\n"
            "    a.stamps[8ull * blockIdx.x + 2] = st2; a.stamps[8ull * blockIdx.x + 3] = __builtin_amdgcn_s_memrealtime(); }\n"
            "  if (!s_last) return;\n  small_compact(a, tab, reinterpret_cast<uint32_t *>(dyn_lds), wtot);\n"
            "  __syncthreads();\n"
            "  if (threadIdx.x == 0) a.stamps[8ull * blockIdx.x + 4] = __builtin_amdgcn_s_memrealtime();\n")
    a = sub(a, "  sa.ctr = ctx->d_small_ctr;\n",
            "  sa.ctr = ctx->d_small_ctr;\n  std::vector<uint64_t> hst;\n"
            "  { uint64_t *d = nullptr; if (hipMalloc((void **)&d, 64ull * nblocks * 5) != hipSuccess) return 1;\n"
            "    (void)hipMemset(d, 0, 64ull * nblocks * 5); sa.stamps = d; hst.resize(40ull * nblocks); }\n")
    a = sub(a, "  const uint64_t nres = hout[0];\n  const KernelSpan spans[1]",
            "  const uint64_t nres = hout[0];\n"
            "  if (getenv(\"RBGPU_SMALL_STAMPS\")) {\n"
            "    (void)hipMemcpy(hst.data(), sa.stamps, 320ull * nblocks, hipMemcpyDeviceToHost);\n"
            "    uint64_t t0 = ~0ull, tw = 0, tc = 0, tcs = 0; uint32_t il = 0;\n"
            "    std::vector<double> al, wk, fin, sr, ky;\n"
            "    for (uint32_t i = 0; i < nblocks; ++i) { const uint64_t *h = &hst[8ull * i]; t0 = std::min(t0, h[0]);\n"
            "      if (h[2] > tw) { tw = h[2]; il = i; } if (h[4]) { tc = h[4]; tcs = h[3]; }\n"
            "      sr.push_back((h[5] - h[0]) / 100.0); ky.push_back((h[6] - h[5]) / 100.0); al.push_back((h[1] - h[6]) / 100.0); wk.push_back((h[2] - h[1]) / 100.0); fin.push_back((h[3] - h[2]) / 100.0); }\n"
            "    uint64_t late = 0; for (uint32_t i = 0; i < nblocks; ++i) late = std::max(late, hst[8ull * i] - t0);\n"
            "    auto pct = [](std::vector<double> v, double q) { std::sort(v.begin(), v.end()); return v[(size_t)(q * (v.size() - 1))]; };\n"
            "    uint32_t pl = 0; for (uint32_t p = 0; p < np; ++p) if ((inl ? (uint32_t)ti->blk[p] : blk[p]) <= il) pl = p;\n"
            "    const uint64_t *h = &hst[8ull * il];\n"
            "    fprintf(stderr, \"stamps blocks %u E %llu kpw %u | last start +%.2f | pair search p50 %.2f max %.2f | keys p50 %.2f max %.2f | align p50 %.2f max %.2f | work p50 %.2f p90 %.2f max %.2f | \"\n"
            "      \"counters p50 %.2f max %.2f | latest work end +%.2f (block %u pair %u nk %u: start +%.2f align %.2f work %.2f) | \"\n"
            "      \"last add +%.2f compaction end +%.2f\\n\", nblocks, (unsigned long long)E, kpw, late / 100.0, pct(sr, .5), pct(sr, 1), pct(ky, .5), pct(ky, 1), pct(al, .5), pct(al, 1),\n"
            "      pct(wk, .5), pct(wk, .9), pct(wk, 1), pct(fin, .5), pct(fin, 1), (tw - t0) / 100.0, il, pl,\n"
            "      (unsigned)(slot[pl + 1] - slot[pl]), (h[0] - t0) / 100.0, (h[1] - h[0]) / 100.0, (h[2] - h[1]) / 100.0,\n"
            "      (tcs - t0) / 100.0, (tc - t0) / 100.0);\n"
            "    for (int w = 0; w < 4; ++w) { const uint64_t *q = &hst[8ull * nblocks + 8ull * (4ull * il + w)];\n"
            "      const unsigned nk_ = (unsigned)(q[4] >> 8);\n"
            "      fprintf(stderr, \"  wave %d: loop start +%.2f, %u keys:\", w, (q[0] - t0) / 100.0, nk_);\n"
            "      for (unsigned k = 0; k < nk_ && k < 3; ++k) fprintf(stderr, \" %s %.2f\", (q[4] >> k) & 1 ? \"M\" : \"C\", (q[1 + k] - (k ? q[k] : q[0])) / 100.0);\n"
            "      if (q[5]) fprintf(stderr, \" | merge key: metadata +%.2f, staged +%.2f, merged+stored +%.2f\", (q[5] - q[0]) / 100.0, (q[6] - q[5]) / 100.0, (q[7] - q[6]) / 100.0);\n"
            "      fprintf(stderr, \"\\n\"); }\n"
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
