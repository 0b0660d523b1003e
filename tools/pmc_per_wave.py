"""Per-wave means of a rocprofv3 --pmc counter_collection.csv, per kernel whose name contains the
filter (SQ counters summed over the dispatch, divided by its SQ_WAVES when collected)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
filt = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    if filt in r["Kernel_Name"]:
        agg[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in agg.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    w = m.get("SQ_WAVES", 1.0)
    print(k, {n: round(v / w, 1) for n, v in sorted(m.items()) if n != "SQ_WAVES"}, "waves", int(w))
