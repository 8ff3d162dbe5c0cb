"""Summarise rocprofv3 --pmc CSVs (gpurun_out/pmc/*) per kernel: mean per dispatch."""
import csv
import collections
import json
import os
import sys

base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for p in sorted(os.listdir(base)):
    f = os.path.join(base, p, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        short = ("jpeg_rgba" if "jpeg_rgba" in name else "jpeg_block" if "jpeg_block_kernel" in name
                 else "png_unfilter" if "png_unfilter" in name
                 else "png_pair" if "png_pair_kernel" in name
                 else "png_adam7_merge" if "png_adam7_merge" in name else None)
        import re
        if short == "png_pair":  # one entry per depth template (tc8 vs the Adam7 RGBA16 line)
            m = re.search(r"png_pair_kernel<(\d+)(?:, *\w+, *(\w+))?", name)
            if m and m.group(1) != "6":
                short = "png_pair_d" + m.group(1)
            if m and m.group(2) == "true":  # the Adam7 pass-6 merge launch
                short += "_merge" if short != "png_pair" else "_d6_merge"
        if short == "jpeg_block":  # the headline instance keeps the plain key
            m = re.search(r"jpeg_block_kernel<([^>]*)>", name)
            if m and m.group(1).replace(" ", "") not in ("signedchar,true,2,2,1,1,0", "char,true,2,2,1,1,0"):
                short = "jpeg_block<" + m.group(1).replace(" ", "") + ">"
        if not short:
            continue
        acc[short][(r["Counter_Name"], r["Dispatch_Id"])].append(float(r["Counter_Value"]))
out = {}
for k, d in acc.items():
    per = collections.defaultdict(list)
    for (cn, disp), vals in d.items():
        per[cn].append(sum(vals))
    out[k] = {cn: sum(v) / len(v) for cn, v in per.items()}
print(json.dumps(out, indent=1))

# roofline.traffic for bench.py: HBM bytes per launch of the fused JPEG kernel,
# FETCH_SIZE/WRITE_SIZE in KiB; FETCH_SIZE doubled (gfx950 tallies a 128-B
# streaming read request as 64 B, MI355X_MICROARCH.md "HBM").
jk = "jpeg_block" if "jpeg_block" in out else "jpeg_rgba"
if len(sys.argv) > 2 and jk in out:
    j = out[jk]
    tr = {"kernel": jk + "_kernel", "images": int(sys.argv[3]) if len(sys.argv) > 3 else 64,
          "size": int(sys.argv[4]) if len(sys.argv) > 4 else 4096,
          "fetch_bytes_per_launch": 2 * j["FETCH_SIZE"] * 1024, "write_bytes_per_launch": j["WRITE_SIZE"] * 1024,
          "note": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950 correction) + WRITE_SIZE, KiB -> B, mean per dispatch"}
    tr["hbm_bytes_per_launch"] = tr["fetch_bytes_per_launch"] + tr["write_bytes_per_launch"]
    try:  # the coefficient transport the passes ran with (bench config)
        tr["coeff_bits"] = json.load(open(os.path.join(base, "fetch.json")))["config"]["coeff_bits"]
    except Exception:
        tr["coeff_bits"] = 16
    # the paired-row PNG kernel reads the band slab (png_slab.cpp): 1 KiB
    # contiguous per load instruction, the streaming shape the x2 is
    # calibrated on (tools/ubench/png_load_pattern mode 2 reads that shape)
    if "png_pair" in out:
        p = out["png_pair"]
        tr["png"] = {"kernel": "png_pair_kernel<TC8>", "images": tr["images"], "size": tr["size"],
                     "fetch_bytes_per_launch": 2 * p["FETCH_SIZE"] * 1024,
                     "write_bytes_per_launch": p["WRITE_SIZE"] * 1024,
                     "note": "FETCH_SIZE x2 (slab loads: 1 KiB contiguous per instruction) + WRITE_SIZE, "
                             "KiB -> B, mean per dispatch"}
        tr["png"]["hbm_bytes_per_launch"] = tr["png"]["fetch_bytes_per_launch"] + tr["png"]["write_bytes_per_launch"]
    if "png_pair_d15" in out and "png_pair_d15_merge" in out:
        a, b = out["png_pair_d15"], out["png_pair_d15_merge"]
        tr["adam7_rgba16"] = {
            "kernel": "png_pair_kernel<TCA16> x2 (passes 1-5 to staging; passes 6-7 merging it)",
            "images": tr["images"], "size": tr["size"],
            "fetch_bytes_per_launch": 2 * (a["FETCH_SIZE"] + b["FETCH_SIZE"]) * 1024,
            "write_bytes_per_launch": (a["WRITE_SIZE"] + b["WRITE_SIZE"]) * 1024,
            "note": "both launches of one plan launch; FETCH_SIZE x2 (slab loads 1 KiB contiguous per "
                    "instruction; pass 6's staging reads 64 B contiguous per 8 lanes) + WRITE_SIZE"}
        t = tr["adam7_rgba16"]
        t["hbm_bytes_per_launch"] = t["fetch_bytes_per_launch"] + t["write_bytes_per_launch"]
    if "png_unfilter" in out:
        p = out["png_unfilter"]
        tr["png_unfilter"] = {"fetch_bytes_per_launch": 2 * p["FETCH_SIZE"] * 1024,
                              "write_bytes_per_launch": p["WRITE_SIZE"] * 1024}
    json.dump(tr, open(sys.argv[2], "w"), indent=1)
