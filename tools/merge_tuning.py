"""Add the entries of a freshly tuned table whose shape keys the committed table does not have
(e.g. SDXL-only shapes), keeping every committed entry as it is.

    python tools/merge_tuning.py NEW.json [--table cassmantle_amd/ops/gemm_tuning.json]
"""
import argparse
import json
import os
import sys

ap = argparse.ArgumentParser()
ap.add_argument("new")
ap.add_argument("--table", default=os.path.join(os.path.dirname(__file__), "..", "cassmantle_amd", "ops", "gemm_tuning.json"))
ap.add_argument("--model", default=None, help="tag the added entries with this model name")
ap.add_argument("--only-cfg", type=int, default=None,
                help="instead: take (and override with) only the new entries whose best plan is this tile config")
a = ap.parse_args()
cur = json.load(open(a.table))
new = json.load(open(a.new))
have = {e["key"] for e in cur["entries"]}
if a.only_cfg is not None:
    take = {e["key"]: e for e in new["entries"] if e["cfg"] == a.only_cfg}
    cur["entries"] = [e for e in cur["entries"] if e["key"] not in take]
    added = list(take.values())
else:
    added = [e for e in new["entries"] if e["key"] not in have]
for e in added:
    if a.model:
        e["model"] = a.model
cur["entries"].extend(added)
json.dump(cur, open(a.table, "w"), indent=1)
print(f"added {len(added)} entries ({len(new['entries']) - len(added)} already present)", file=sys.stderr)
