"""Digest of an ab_loaders.py JSONL: per case, the sorted times of each setting and identity."""
import collections
import json
import sys

d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    r = json.loads(line)
    if "us" in r:
        d[(r["path"], r["shape"], r["cfg"], r.get("set", r.get("loaders")))].append(r["us"])
    elif not r.get("bit_identical", True):
        print("NOT bit-identical:", r)
for k, v in d.items():
    print(*k, sorted(v))
