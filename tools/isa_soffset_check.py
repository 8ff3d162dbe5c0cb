"""ISA audit of the library's buffer instructions (round-5 verdict item 4):
every MUBUF load / store of every kernel must take soffset 0.  A raw
buffer's range check leaves soffset out (the b9be61c bug: an offset carried
in soffset let a prefetch past a band's last group read the bytes after the
stream instead of zeros), so the kernels put the whole offset in voffset and
rely on the check for out-of-range zeros / dropped stores.

Compiles each .hip source of zpix_amd/csrc to gfx950 assembly (device only)
and lists every buffer_* instruction whose soffset operand is not 0.
Usage: python tools/isa_soffset_check.py   (exit 1 on a finding)"""
import concurrent.futures as cf
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "zpix_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def isa(src, out):
    subprocess.run([HIPCC, "--offload-arch=gfx950", "--cuda-device-only", "-S", "-O3", "-std=c++17", "-fwrapv",
                    "-I", os.path.join(ROOT, "include"), "-I", CSRC, src, "-o", out], check=True)
    return out


def main():
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    bad = 0
    total = 0
    with tempfile.TemporaryDirectory() as d, cf.ThreadPoolExecutor(8) as ex:
        outs = list(ex.map(lambda s: isa(s, os.path.join(d, os.path.basename(s) + ".s")), srcs))
        for src, out in zip(srcs, outs):
            fn = None
            for line in open(out):
                m = re.match(r"^(\S+):\s*(;.*)?$", line)
                if m and not m.group(1).startswith("."):
                    fn = m.group(1)
                t = line.strip()
                if not t.startswith("buffer_") or t.startswith(("buffer_inv", "buffer_wbl2", "buffer_wbinvl1")):
                    continue
                total += 1
                ops = [o.strip() for o in t.split(None, 1)[1].split(",")]
                # buffer_load/store vdata, vaddr|off, srsrc, soffset [modifiers]
                so = ops[3].split()[0] if len(ops) > 3 else "?"
                if so not in ("0", "off"):
                    bad += 1
                    print(f"{os.path.basename(src)}: {fn}: {t}")
    print(f"{total} buffer instructions, {bad} with a nonzero soffset")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
