"""Static VALU cost of the render kernel per code section (analysis aid).

Builds vr_render.hip to assembly with -DVR_MARKS (asm ';@mark <name>' comments at the section
starts of vr_render.hip), takes the C3 kernel (render_kernel<32, false, false, true, 1, 3, false>),
attributes every instruction to the last marker above it in layout order, and prices each
instruction with a simple gfx950 issue model (wave64: f32 / int VALU 2 cycles, f64 and 64-bit ops 4,
f64 transcendentals 16, 32-bit integer multiplies 8).
    python tools/isa_sections.py [extra hipcc flags]"""
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the C3 timed kernel: STACK 32, Lambertian-only, DARK0, no Whitted, no cooperative tail (VR_ISA_STACK /
# VR_ISA_MATS / VR_ISA_COOP=1 pick another instantiation)
KERNEL = ("_ZN2vr3dev13render_kernelILi%sELb0ELb0ELb1ELi%sELi3ELb0ELb%sELb0EEEvNS_10RenderArgsEPKNS_4PrimEPKNS_8MaterialEPKNS_3BvhE"
          % (os.environ.get("VR_ISA_STACK", "32"), os.environ.get("VR_ISA_MATS", "1"), os.environ.get("VR_ISA_COOP", "0")))


def cost(op):
    if not op.startswith("v_"):
        return 0
    if re.match(r"v_(rcp|rsq|sqrt|exp|log|sin|cos|frexp_mant|frexp_exp)_f64", op):
        return 16
    if "f64" in op or "_u64" in op or "_i64" in op or "b64" in op and op.startswith("v_lshl") or op.startswith("v_pk_"):
        return 4
    if re.match(r"v_mul_(lo|hi)_(u|i)32|v_mad_(u|i)64", op):
        return 8
    return 2


def main():
    out = os.path.join(tempfile.mkdtemp(), "render.s")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
           "-fno-fast-math", "--cuda-device-only", "-S", "-DVR_MARKS"] + sys.argv[1:] + \
          [os.path.join(ROOT, "vanrijn_amd/csrc/vr_render.hip"), "-o", out]
    subprocess.check_call(cmd, stderr=subprocess.DEVNULL)
    lines = open(out).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(KERNEL + ":"))
    sec = "entry"
    stats = collections.defaultdict(lambda: collections.Counter())
    ops = collections.defaultdict(lambda: collections.Counter())
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        m = re.search(r";@mark (\w+)", l)
        if m:
            sec = m.group(1)
            continue
        t = l.strip()
        if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
            continue
        op = t.split()[0]
        st = stats[sec]
        st["insts"] += 1
        ops[sec][op] += 1
        if op.startswith("v_"):
            st["valu"] += 1
            st["cycles"] += cost(op)
            if "f64" in op:
                st["f64"] += 1
        elif op.startswith("s_"):
            st["salu"] += 1
        if op.startswith(("global_", "buffer_", "flat_")):
            st["vmem"] += 1
        if op.startswith("ds_"):
            st["lds"] += 1
    print("%-14s %6s %6s %6s %6s %7s %5s %5s" % ("section", "insts", "valu", "f64", "salu", "vcycles", "vmem", "lds"))
    for k, st in stats.items():
        print("%-14s %6d %6d %6d %6d %7d %5d %5d" % (k, st["insts"], st["valu"], st["f64"], st["salu"], st["cycles"],
                                                    st["vmem"], st["lds"]))
    for k in os.environ.get("VR_ISA_OPS", "").split(","):  # opcode histograms of these sections
        if k in ops:
            print("\n" + k + ": " + ", ".join("%s %d" % kv for kv in ops[k].most_common() if kv[0].startswith("v_")))


if __name__ == "__main__":
    main()
