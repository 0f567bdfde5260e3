"""Summarise a tools/gpu_ab_env.sh log: per (line, setting) the host median, graph and record
path of each round.    python tools/ab_summary.py gpurun_out/TAG_steps.jsonl"""
import collections
import json
import sys

acc = collections.defaultdict(list)
m = None
for line in open(sys.argv[1]):
    if line.startswith("=="):
        m = line.split()[-1]
        continue
    try:
        d = json.loads(line)
    except ValueError:
        continue
    for k, v in d.items():
        acc[(k, m)].append((v.get("dropin_step_us_median"), v.get("graph_replay_us"),
                            v.get("record_path_latency_us")))
for k, v in sorted(acc.items()):
    print(k, v)
