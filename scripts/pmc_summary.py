"""Summarize rocprofv3 --pmc CSVs: per kernel name, mean counter value per dispatch."""
import csv, glob, sys, collections
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        name = row["Kernel_Name"].split("(")[0].replace("void ", "")
        agg[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
        agg[name]["_dur_ns"].append(float(row["End_Timestamp"]) - float(row["Start_Timestamp"]))
for name, cs in agg.items():
    if not any(k in name for k in sys.argv[2:] or [""]):
        continue
    print(name)
    for k, v in sorted(cs.items()):
        print(f"   {k:28s} {sum(v)/len(v):16.1f}  (n={len(v)})")
