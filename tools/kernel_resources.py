"""VGPR / SGPR / scratch / LDS of the render-kernel instantiations (analysis aid).
    python tools/kernel_resources.py [extra hipcc flags]"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    out = os.path.join(tempfile.mkdtemp(), "render.s")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                           "-ffp-contract=off", "-fno-fast-math", "--cuda-device-only", "-S"] + sys.argv[1:] +
                          [os.path.join(ROOT, "vanrijn_amd/csrc/vr_render.hip"), "-o", out], stderr=subprocess.DEVNULL)
    meta = open(out).read().split("amdhsa.kernels:")[1]
    for blk in re.split(r"\n  - ", meta):
        name = re.search(r"\.name:\s+(\S+)", blk)
        if not name or "render_kernel" not in name.group(1):
            continue
        args = re.search(r"render_kernelIL(.*?)EEEv", name.group(1)).group(1)
        f = {k: re.search(r"\." + k + r":\s+(\d+)", blk) for k in
             ("vgpr_count", "sgpr_count", "sgpr_spill_count", "vgpr_spill_count", "private_segment_fixed_size",
              "group_segment_fixed_size")}
        print("%-40s vgpr %3s sgpr %3s sgpr_spill %3s scratch %4s lds %6s" % (
            args, f["vgpr_count"].group(1), f["sgpr_count"].group(1), f["sgpr_spill_count"].group(1),
            f["private_segment_fixed_size"].group(1), f["group_segment_fixed_size"].group(1)))


if __name__ == "__main__":
    main()
