#!/usr/bin/env python3
"""merge_pmc_legs.py <prof_legs dir> ... — fold profile_legs.sh summaries
(<dir>/pmc_legs.json, keyed "<workload key>|<leg>") into profiles/pmc_legs.json, the
table bench.py reads its per-leg `traffic` from; later directories win."""
import json
import os
import sys

DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "pmc_legs.json")
table = json.load(open(DST)) if os.path.exists(DST) else {}
for d in sys.argv[1:]:
    part = json.load(open(os.path.join(d, "pmc_legs.json")))
    table.update(part)
    print("%s: %d entries" % (d, len(part)))
with open(DST, "w") as f:
    json.dump(dict(sorted(table.items())), f, indent=1)
print("%s: %d entries" % (DST, len(table)))
