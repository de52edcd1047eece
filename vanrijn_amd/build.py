"""Build the in-tree HIP library vanrijn_amd/lib/libvanrijn_amd.so for gfx950 (hipcc)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB_DIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIB_DIR, "libvanrijn_amd.so")
SOURCES = ["vr_render.hip", "vr_image.hip", "vr_build.hip", "vr_host.cpp"]
HEADERS = ["vr_layout.h", "vr_device.h", "rgb_spectrum_tables.h", "vr_exp_table.h", os.path.join("..", "..", "include", "vanrijn_amd.h")]

FLAGS = [
    "--offload-arch=gfx950",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-shared",
    # Rust never contracts a*b+c into an FMA; neither may we
    "-ffp-contract=off",
    "-fno-fast-math",
    "-Wall",
    # the AMDGPU register-pressure trackers in the machine scheduler: the same registers (168, no
    # scratch) and bit-identical records, C3's render kernel 37.49 -> 37.06 ms (-1.2 %), C5 -0.2 %
    # (profiles/r06/sched/)
    "-Xarch_device",
    "-mllvm=-amdgpu-use-amdgpu-trackers",
]


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.isabs(c) and os.path.exists(c) or not os.path.isabs(c)):
            return c
    return "hipcc"


def stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    for f in SOURCES + HEADERS:
        if os.path.getmtime(os.path.join(CSRC, f)) > t:
            return True
    return os.path.getmtime(os.path.abspath(__file__)) > t  # the flags changed


def build(force=False, verbose=False):
    """Each source compiles to its own object in parallel (no device-side linking is needed: every
    kernel is launched from its own translation unit), then one shared-library link."""
    if not force and not stale():
        return LIB
    os.makedirs(LIB_DIR, exist_ok=True)
    compile_flags = [f for f in FLAGS if f != "-shared"]
    if os.environ.get("VR_TUNING") == "1":  # the occupancy-variant kernels of tools/variants.py
        compile_flags.append("-DVR_TUNING_VARIANTS")
    objs, procs = [], []
    for src in SOURCES:
        obj = os.path.join(LIB_DIR, os.path.splitext(src)[0] + ".o")
        cmd = [hipcc()] + compile_flags + ["-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append((subprocess.Popen(cmd), cmd))
        objs.append(obj)
    failed = [cmd for p, cmd in procs if p.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])
    link = [hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC"] + objs + ["-lz", "-o", LIB + ".tmp"]
    if verbose:
        print(" ".join(link))
    subprocess.check_call(link)
    for o in objs:
        os.remove(o)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(LIB)
