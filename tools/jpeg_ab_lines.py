"""Kernel ms per launch of every JPEG line in bench.py JSON files (A/B logs):
headline, int16, planar int8/int16, pieces rgba/planes, progressive 4:4:4.
Usage: python tools/jpeg_ab_lines.py <json>..."""
import json
import sys

print("file headline int16 planar8 planar16 pieces.rgba pieces.planes prog444")
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    g = lambda *ks: (lambda v: v)(__import__("functools").reduce(lambda a, k: (a or {}).get(k), ks, d))
    print(f.split("gpurun_out/")[-1], g("roofline", "kernel_ms_per_launch"), g("int16_transport", "kernel_ms_per_launch"),
          g("planar", "int8", "kernel_ms_per_launch"), g("planar", "int16", "kernel_ms_per_launch"),
          g("pieces", "rgba", "kernel_ms_per_launch"), g("pieces", "planes", "kernel_ms_per_launch"),
          g("config5", "jpeg_progressive_444", "kernel_ms_per_launch"))
