"""One line of kernel ms per bench.py line from a bench JSON (A/B output)."""
import json
import sys


def walk(d, path=""):
    for k, v in d.items():
        if isinstance(v, dict):
            if "kernel_ms_per_launch" in v:
                yield (path + k, v["kernel_ms_per_launch"])
            yield from walk(v, path + k + ".")


d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
out = [("headline", d["roofline"]["kernel_ms_per_launch"])] if "roofline" in d and "kernel_ms_per_launch" in d["roofline"] else []
out += [(k, v) for k, v in walk(d) if k != "roofline"]
print(" ".join(f"{k}={v}" for k, v in out))
