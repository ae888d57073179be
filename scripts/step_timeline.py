"""One config-2 step as a timeline from a rocprofv3 kernel trace: every dispatch between two
consecutive headline light-task launches, with its start offset, duration and the idle gap before
it.  usage: python scripts/step_timeline.py <run_kernel_trace.csv>"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ev = [(r["Kernel_Name"].split("(")[0].replace("void ", "").replace("rbg::", ""), int(r["Grid_Size_X"]),
       int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
big = [i for i, e in enumerate(ev) if e[0].startswith("k_pair_tasks<0, false, 0>") and e[3] - e[2] > 1_000_000]
if len(big) < 3:
    sys.exit("need >= 3 headline steps in the trace")
a, b = big[-3], big[-2]  # a step from the end of one headline task phase to the next
t_end = max(e[3] for e in ev[a:a + 2])
start = ev[a][2]
print(f"{'kernel':42s} {'grid':>9s} {'start_us':>9s} {'dur_us':>9s} {'gap_us':>8s}")
prev_end = ev[a][2]
for e in ev[a:b]:
    print(f"{e[0][:42]:42s} {e[1]:9d} {(e[2] - start) / 1e3:9.1f} {(e[3] - e[2]) / 1e3:9.1f} "
          f"{max(0, e[2] - prev_end) / 1e3:8.1f}")
    prev_end = max(prev_end, e[3])
print(f"step span (task start to next task start): {(ev[b][2] - start) / 1e3:.1f} us")
