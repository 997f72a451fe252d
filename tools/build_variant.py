"""Build an in-tree variant of libmvmatch.so with extra -D macros for A/B
timing (tools/ab_same_buffers.py, tools/gpu.sh ab): the library's own build
flags plus the macros, written to bpc_baseline_amd/lib/ab/<name>.so.

python tools/build_variant.py NAME [MACRO[=VALUE] ...]
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as G  # noqa: E402

name, macros = sys.argv[1], sys.argv[2:]
out_dir = os.path.join(G.LIB_DIR, "ab")
os.makedirs(out_dir, exist_ok=True)
out = os.path.join(out_dir, name + ".so")
subprocess.run([G._hipcc(), *G.HIPCC_FLAGS, "-I" + os.path.join(G.PKG, "csrc"),
                *("-D" + m for m in macros), "-o", out, *G.HIP_SRCS], check=True)
print(out)
