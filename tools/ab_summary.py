"""Summarise tools/lib_ab.sh output: best and mean us/generation per (board, library), with every round."""
import collections
import json
import sys

d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    r = json.loads(line)
    if "us_per_gen" in r:
        d[(r["w"], r["h"], r["boundary"], r.get("variant", ""), r["lib"])].append(r["us_per_gen"])
for k in sorted(d):
    v = d[k]
    print(k, "best %.4f mean %.4f" % (min(v), sum(v) / len(v)), v)
