"""Summary of scripts/rehearse_n2.sh: per workload the N=1 and N=2 lines' global results."""
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/n2"


def last_json(path):
    for line in reversed(open(path).read().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    return None


KEYS = ("result_cardinality", "result_cardinality_all_ranks", "result_serialized_bytes")
for f1 in sorted(glob.glob(os.path.join(root, "*_n1.json"))):
    w = os.path.basename(f1)[:-8]
    a, b = last_json(f1), last_json(f1.replace("_n1.json", "_n2.json"))
    if a is None or b is None:
        print(w, "missing line")
        continue
    ca = {k: a["config"][k] for k in KEYS if k in a["config"]}
    cb = {k: b["config"][k] for k in KEYS if k in b["config"]}
    card = [d.get("result_cardinality", d.get("result_cardinality_all_ranks")) for d in (ca, cb)]
    same = ("weak: each rank its own pairs" if b["scaling"] == "weak"
            else "same global cardinality" if card[0] == card[1] else "CARDINALITY DIFFERS")
    print(f"{w}: n1 {a['value']} {a['unit']} n2 {b['value']} (n_gpus {b['n_gpus']}, scaling {b['scaling']}) "
          f"result n1 {ca} n2 {cb} -> {same}")
