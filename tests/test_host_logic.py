"""Host-side planning logic of the PNG/JPEG paths, without a GPU: the band
schedule's no-deadlock order and longest-first rule, the Adam7 staging layout
and merge jobs, and the block kernel's quant-pair tables
(tests/host_logic_check.cpp, linked against libzpix_amd.so)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_png_schedule_adam7_stage_and_quant_pairs(tmp_path):
    lib_dir = os.path.join(ROOT, "zpix_amd")
    if not os.path.exists(os.path.join(lib_dir, "libzpix_amd.so")):
        pytest.skip("libzpix_amd.so not built")
    exe = str(tmp_path / "host_logic_check")
    subprocess.run([HIPCC, "-O1", "-std=c++17", "-I", os.path.join(ROOT, "include"),
                    "-I", os.path.join(ROOT, "zpix_amd", "csrc"), os.path.join(ROOT, "tests", "host_logic_check.cpp"),
                    "-L", lib_dir, "-lzpix_amd", f"-Wl,-rpath,{lib_dir}", "-o", exe], check=True, timeout=300)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr
