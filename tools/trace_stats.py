"""Per-launch-shape kernel statistics from a rocprofv3 kernel trace.

rocprofv3 --stats averages every dispatch of a kernel together, and bench.py
launches the same template both over the 64-frame batch (the headline) and
per image (the end-to-end line), so its per-kernel average mixes the two.
This groups the trace by (kernel, stream, grid size) instead; bench.py
times the batch launches on a stream of their own, so the headline
launch's average can be compared with bench.py's HIP-event figure.

Warm-up launches are dropped: within each (kernel, stream, grid) group the
first `--skip-first` launches (default 5, >= bench.py's warm-up count of
every timed line) are left out, so the averages describe timed launches
only (a group with no more launches than that keeps its last one).

usage: python tools/trace_stats.py run_kernel_trace.csv [--skip-first N] > by_launch.csv
"""
import csv
import re
import sys
from collections import defaultdict


def short_name(name: str) -> str:
    name = re.sub(r"zpx::\(anonymous namespace\)::", "", name)
    return re.sub(r"\(.*\)$", "", name).replace("void ", "")


def main(path: str, skip: int) -> None:
    groups = defaultdict(list)
    with open(path, newline="") as f:
        rows = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))  # launch order
        for row in rows:
            key = (short_name(row["Kernel_Name"]), int(row["Stream_Id"]), int(row["Grid_Size_X"]),
                   int(row["Workgroup_Size_X"]))
            groups[key].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6)
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "stream", "grid_x", "workgroup_x", "calls", "skipped", "avg_ms", "median_ms", "min_ms",
                "max_ms", "total_ms"])
    for key, d in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        k = min(skip, len(d) - 1)
        t = d[k:]
        med = sorted(t)[len(t) // 2]
        w.writerow([*key, len(t), k, f"{sum(t) / len(t):.4f}", f"{med:.4f}", f"{min(t):.4f}", f"{max(t):.4f}",
                    f"{sum(t):.3f}"])


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip-first", type=int, default=5)
    a = ap.parse_args()
    main(a.trace, a.skip_first)
