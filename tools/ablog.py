#!/usr/bin/env python3
"""Summarize a gpu_session A/B log of tools/round_probe.py runs ("== label" lines followed by per-round JSON)."""
import json
import sys

cur, res = None, {}
for line in open(sys.argv[1]):
    if line.startswith("=="):
        cur = line[3:].strip()
        res[cur] = []
    elif line.startswith('{"round"'):
        res[cur].append(json.loads(line)["kernel_ms"])
for k, v in res.items():
    print(f"{k:24s} tot={sum(v):.3f} " + " ".join(f"{x:.3f}" for x in v))
