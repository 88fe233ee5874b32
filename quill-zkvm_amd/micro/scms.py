"""print the sumcheck ms fields of bench JSON logs: python scms.py <log>..."""
import json
import sys


def find(x):
    if isinstance(x, dict):
        if "round_kernels_ms_per_call" in x:
            return x
        for v in x.values():
            r = find(v)
            if r:
                return r
    return None


for f in sys.argv[1:]:
    for line in open(f):
        if line.startswith("{"):
            d = find(json.loads(line))
            print(f, {k: round(v, 4) for k, v in d.items() if "ms" in k})
