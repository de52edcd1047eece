"""Compare the gfx950 ISA of vr_render.hip's kernels between two builds (refactoring check).

    python tools/isa_diff.py save BEFORE.s     # device assembly of the current source
    python tools/isa_diff.py diff BEFORE.s     # rebuild and list kernels whose instructions differ
Extra hipcc flags may follow the file name.  Comments, directives and labels' names are ignored;
kernel-argument offsets and register numbers are compared as written."""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
         "--cuda-device-only", "-S"]


def build(out, extra):
    subprocess.check_call(["/opt/rocm/bin/hipcc"] + FLAGS + extra +
                          [os.path.join(ROOT, "vanrijn_amd/csrc/vr_render.hip"), "-o", out], stderr=subprocess.DEVNULL)


def kernels(path):
    out, cur = {}, None
    for line in open(path).read().split("\n"):
        m = re.match(r"^([_A-Za-z0-9]+):", line)
        if m and m.group(1).startswith("_ZN2vr3dev"):
            cur = m.group(1)
            out[cur] = []
            continue
        if cur is None:
            continue
        if line.startswith(".Lfunc_end"):
            cur = None
            continue
        t = line.split(";")[0].strip()
        if not t or t.startswith(".") or t.endswith(":"):
            continue
        out[cur].append(re.sub(r"\.LBB\d+_\d+", "L", t))
    return out


def main():
    mode, path, extra = sys.argv[1], sys.argv[2], sys.argv[3:]
    if mode == "save":
        build(path, extra)
        return
    now = os.path.join(tempfile.mkdtemp(), "now.s")
    build(now, extra)
    a, b = kernels(path), kernels(now)
    same = 0
    for k in sorted(set(a) | set(b)):
        if a.get(k) == b.get(k):
            same += 1
        else:
            print("DIFF %-90s %6s -> %6s instructions" % (k[:90], len(a.get(k, [])), len(b.get(k, []))))
    print("%d kernels, %d identical" % (len(set(a) | set(b)), same))


if __name__ == "__main__":
    main()
