"""Build a diagnostic library variant quickly: the product build's objects are reused for every
source except the ones named (recompiled with the extra defines) and runtime.hip (build id).

usage: python scripts/variant_build.py <variant> <DEFINE[=v]>[,DEFINE...] <src.hip>[,src.hip...]
   -> video-spike_amd/vspike/_build/libvspike_<variant>.so  (select with VSPIKE_LIB=...)
"""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-spike_amd"))
from vspike import build  # noqa: E402


def main(variant, defines, srcs):
    if not os.environ.get("VB_NO_PRODUCT"):  # (VB_NO_PRODUCT=1: leave libvspike.so alone, e.g. while a
        build.build(verbose=False)           # GPU call that ships it is pending)
    vdir = os.path.join(build.BUILD_DIR, variant)
    os.makedirs(vdir, exist_ok=True)
    redo = {os.path.splitext(s)[0] + ".o" for s in srcs} | {"runtime.o"}
    for f in os.listdir(build.BUILD_DIR):
        if f.endswith(".o"):
            dst = os.path.join(vdir, f)
            if f in redo:
                if os.path.exists(dst):
                    os.remove(dst)
            else:
                shutil.copy2(os.path.join(build.BUILD_DIR, f), dst)
                os.utime(dst)  # newer than every source: not recompiled
    return build.build(variant=variant, defines=defines, verbose=True)


if __name__ == "__main__":
    print(main(sys.argv[1], [d for d in sys.argv[2].split(",") if d], sys.argv[3].split(",")))
