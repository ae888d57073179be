"""Per-(kernel, grid) dispatch groups of a rocprofv3 kernel trace: count, average and min duration,
and for concurrent pairs the union span of overlapping dispatches.  The bench's headline launch is
one group (one grid size); --stats averages every dispatch of a kernel, including the small
secondary / CPU-baseline-sample calls of the same kernel.
usage: python scripts/trace_groups.py <run_kernel_trace.csv> [name-substring ...]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
subs = sys.argv[2:]
groups = collections.defaultdict(list)
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if subs and not any(s in name for s in subs):
        continue
    grid = int(r["Grid_Size_X"])
    groups[(name, grid)].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
print(f"{'kernel':45s} {'grid':>9s} {'n':>4s} {'avg_ms':>9s} {'min_ms':>9s} {'big_n':>5s} {'big_avg_ms':>10s}")
for (name, grid), d in sorted(groups.items(), key=lambda kv: -sum(e - s for s, e in kv[1])):
    durs = [(e - s) / 1e6 for s, e in d]
    big = [x for x in durs if x >= 0.5 * max(durs)]  # the headline-size dispatches of the group
    print(f"{name:45s} {grid:9d} {len(d):4d} {sum(durs) / len(durs):9.4f} {min(durs):9.4f} {len(big):5d} "
          f"{sum(big) / len(big):10.4f}")
# union spans of one call's task phase, per op (the template's first argument: 0 AND, 1 OR, 2 XOR,
# 3 ANDNOT): every light and heavy dispatch of the op, clustered by overlap (a dispatch that starts
# within 50 us of the cluster's end joins it), so the two launches of each kind count once per call
OPS = {"0": "AND", "1": "OR", "2": "XOR", "3": "ANDNOT"}
for opk, opname in OPS.items():
    ds = sorted(x for (n, g), v in groups.items() if "k_pair_tasks<" + opk + "," in n for x in v)
    spans, cur = [], None
    for st, en in ds:
        if cur and st <= cur[1] + 50_000:
            cur[1] = max(cur[1], en)
        else:
            if cur:
                spans.append((cur[1] - cur[0]) / 1e6)
            cur = [st, en]
    if cur:
        spans.append((cur[1] - cur[0]) / 1e6)
    if not spans:
        continue
    big = sorted(x for x in spans if x >= 0.5 * max(spans))
    med = big[len(big) // 2]
    print(f"{opname:6s} task-phase union spans (headline-size calls): n={len(big)} median_ms={med:.4f} "
          f"avg_ms={sum(big) / len(big):.4f} min_ms={min(big):.4f} max_ms={max(big):.4f}")
