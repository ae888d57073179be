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
# union spans of the concurrent light/heavy pair (dispatches that overlap in time)
lt = sorted(x for (n, g), v in groups.items() if n.endswith("0>") and "k_pair_tasks" in n for x in v)
hv = sorted(x for (n, g), v in groups.items() if n.endswith("1>") and "k_pair_tasks" in n for x in v)
spans = []
for s2, e2 in hv:
    # the light launch beside the heavy kernel, and the second light launch that starts on the side
    # stream when the heavy kernel ends (both take tasks from one queue)
    ph = [(s, e) for s, e in lt if s < e2 + 50_000 and e > s2]
    if ph:
        spans.append((max([e2] + [e for _, e in ph]) - min([s2] + [s for s, _ in ph])) / 1e6)
if spans:
    big = [x for x in spans if x >= 0.5 * max(spans)]
    print(f"  headline-size spans: n={len(big)} avg_ms={sum(big) / len(big):.4f}")
    print(f"concurrent light||heavy union spans: n={len(spans)} avg_ms={sum(spans) / len(spans):.4f} "
          f"min_ms={min(spans):.4f}")
