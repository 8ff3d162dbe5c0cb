"""Per-launch-shape kernel statistics from a rocprofv3 kernel trace.

rocprofv3 --stats averages every dispatch of a kernel together, and bench.py
launches the same template both over the 64-frame batch (the headline) and
per image (the end-to-end line), so its per-kernel average mixes the two.
This groups the trace by (kernel, stream, grid size) instead; bench.py
times the batch launches on a stream of their own, so the headline
launch's average can be compared with bench.py's HIP-event figure.

usage: python tools/trace_stats.py run_kernel_trace.csv > by_launch.csv
"""
import csv
import re
import sys
from collections import defaultdict


def short_name(name: str) -> str:
    name = re.sub(r"zpx::\(anonymous namespace\)::", "", name)
    return re.sub(r"\(.*\)$", "", name).replace("void ", "")


def main(path: str) -> None:
    groups = defaultdict(list)
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            key = (short_name(row["Kernel_Name"]), int(row["Stream_Id"]), int(row["Grid_Size_X"]),
                   int(row["Workgroup_Size_X"]))
            groups[key].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6)
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "stream", "grid_x", "workgroup_x", "calls", "avg_ms", "min_ms", "max_ms", "total_ms"])
    for key, d in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([*key, len(d), f"{sum(d) / len(d):.4f}", f"{min(d):.4f}", f"{max(d):.4f}", f"{sum(d):.3f}"])


if __name__ == "__main__":
    main(sys.argv[1])
