"""Summarise rocprofv3 --pmc CSVs (one directory per pass) per kernel
instance: mean counter value per dispatch; optionally write the HBM
traffic per launch that bench.py reports as roofline.traffic.

Usage: python3 tools/pmc_summary.py <pass dir root> [traffic.json out] [images] [size]

Per kernel instance, each counter is the median over its dispatches of the
per-dispatch total (the bench's batch launches outnumber its small check
launches of the same instance).

HBM bytes: FETCH_SIZE x 2 (gfx950 tallies a 128-B streaming read request as
64 B, MI355X_MICROARCH.md "HBM") + WRITE_SIZE, both in KiB.  A bench line
whose plan runs several kernels (Adam7: two launches of the paired-row
kernel; PNG from the stream: the slab build + the paired-row kernel) sums
them."""
import collections
import csv
import json
import os
import re
import sys

# kernel-name pattern -> short key (the first match wins)
KEYS = [
    # (the block kernels' last template argument: ZPX_COEFFS_PIECES instances)
    (r"jpeg_plane_block_kernel<signed char, false>", "jpeg_plane_block_i8"),
    (r"jpeg_plane_block_kernel<short, false>", "jpeg_plane_block_i16"),
    (r"jpeg_plane_block_kernel<signed char, true>", "jpeg_plane_block_i8_pieces"),
    (r"jpeg_plane_block_kernel<short, true>", "jpeg_plane_block_i16_pieces"),
    (r"jpeg_block_kernel<signed char, true, 2, 2, 1, 1, 0, true>", "jpeg_block_pieces"),
    (r"jpeg_block_kernel<signed char, true, 2, 2, 1, 1, 0, false>", "jpeg_block"),  # the headline instance
    (r"jpeg_block_kernel<short, true, 2, 2, 1, 1, 0, false>", "jpeg_block_i16"),
    (r"jpeg_block_kernel<signed char, true, 1, 1, 1, 1, 0, false>", "jpeg_block_444_i8"),
    (r"jpeg_block_kernel<short, true, 1, 1, 1, 1, 0, false>", "jpeg_block_444_i16"),
    (r"jpeg_block_kernel<([^>]*)>", None),
    (r"jpeg_rgba_kernel", "jpeg_rgba"),
    (r"png_slab_kernel<(\d+)>", "png_slab_cb{0}"),
    (r"png_pair_kernel<(\d+), (\w+), (\w+), (\w+)>", "png_pair_d{0}{2}{3}"),
    (r"png_unfilter_kernel", "png_unfilter"),
    (r"rgba_batch_kernel<6>", "rgba_pixels"),  # (NRGBA64, the bench's rgbaPixels line)
    (r"rgba_pixels_kernel", "rgba_pixels_generic"),
    (r"jpeg_sparse_expand", "jpeg_sparse_expand"),
    (r"jpeg_pieces_expand", "jpeg_pieces_expand"),
]


def short_name(name):
    for pat, key in KEYS:
        m = re.search(pat, name)
        if m:
            if key is None:
                return "jpeg_block<" + m.group(1).replace(" ", "") + ">"
            g = m.groups()
            if key.startswith("png_pair"):
                return "png_pair_d{}{}{}".format(g[0], "_merge" if g[2] == "true" else "",
                                                 "_stream" if g[3] == "true" else "")
            return key.format(*g)
    return None


def summarise(base):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in sorted(os.listdir(base)):
        f = os.path.join(base, p, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            short = short_name(r["Kernel_Name"])
            if short:
                acc[short][(r["Counter_Name"], r["Dispatch_Id"])].append(float(r["Counter_Value"]))
    # per kernel instance and counter: the MEDIAN over its dispatches of the
    # per-dispatch total.  (A run's parity gates and single-image checks
    # launch the same instance on far smaller plans; a mean over all
    # dispatches mixed them in -- Adam7 RGBA16 read 19.6 GB a launch that
    # way, 23.5 with the median.)
    out = {}
    for k, d in acc.items():
        per = collections.defaultdict(list)
        for (cn, _), vals in d.items():
            per[cn].append(sum(vals))
        out[k] = {cn: sorted(v)[len(v) // 2] for cn, v in per.items()}
        out[k]["dispatches"] = max(len(v) for v in per.values())
    return out


# FETCH_SIZE -> bytes read per kernel: x2, the guide's gfx950 correction
# for streaming reads (a 128-B request tallied as 64 B), calibrated for
# 16-B-per-lane coalesced loads.  The paired-row kernel's stream instance
# reads each row's unaligned 96-128-B window on consecutive lanes; its
# figure is the same correction, an upper bound for that shape (requests
# that fetch 64 B are tallied in full).
FETCH_SCALE = {}


def hbm(out, *keys):
    if not all(k in out and "FETCH_SIZE" in out[k] and "WRITE_SIZE" in out[k] for k in keys):
        return None
    f = sum(FETCH_SCALE.get(k, 2) * out[k]["FETCH_SIZE"] * 1024 for k in keys)
    w = sum(out[k]["WRITE_SIZE"] * 1024 for k in keys)
    return {"fetch_bytes_per_launch": f, "write_bytes_per_launch": w, "hbm_bytes_per_launch": f + w,
            "kernels": list(keys)}


# bench.py line -> the kernels one launch of its plan runs
LINES = {
    "headline": ("jpeg_block",),
    "int16": ("jpeg_block_i16",),
    "progressive_444": ("jpeg_block_444_i8",),
    "planar_int8": ("jpeg_plane_block_i8",),
    "planar_int16": ("jpeg_plane_block_i16",),
    "png_stream": ("png_pair_d6_stream",),  # the png line (from the inflated stream)
    "png_slab_input": ("png_pair_d6",),
    "png_slab_build": ("png_slab_cb12",),
    "adam7_rgba16_stream": ("png_pair_d15_stream", "png_pair_d15_merge_stream"),  # the Adam7 line
    "adam7_rgba16_slab_input": ("png_pair_d15", "png_pair_d15_merge"),
    "rgba_pixels_nrgba64": ("rgba_pixels",),
    "pieces_rgba": ("jpeg_block_pieces",),
    "pieces_planes": ("jpeg_plane_block_i8_pieces",),
}

if __name__ == "__main__":
    base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    out = summarise(base)
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 2:
        images = int(sys.argv[3]) if len(sys.argv) > 3 else 64
        size = int(sys.argv[4]) if len(sys.argv) > 4 else 4096
        tr = {"images": images, "size": size,
              "note": "rocprofv3 --pmc, one pass per counter set: FETCH_SIZE x2 (gfx950 correction) + "
                      "WRITE_SIZE, KiB -> B, mean per dispatch, summed over the kernels of one plan launch"}
        for line, keys in LINES.items():
            t = hbm(out, *keys)
            if t:
                tr[line] = t
        json.dump(tr, open(sys.argv[2], "w"), indent=1)
