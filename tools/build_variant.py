"""Build an in-tree variant of libmvmatch.so for A/B timing (tools/ab_same_buffers.py,
tools/gpu.sh ab): the library's own sources and flags, plus diagnostic patches
from tools/diag/ and extra -D macros, written to bpc_baseline_amd/lib/ab/<name>.so.

python tools/build_variant.py NAME [--patch DIAG ...] [MACRO[=VALUE] ...]

The shipped sources carry no diagnostic code path: a patch (e.g. ``no_arith``:
the pairwise stores without the pair arithmetic; ``cheap_lines``: lines not
normalised; ``no_assoc``: no group-end association; ``occ3_c3``: a 640-column
LDS tile reused) is applied to a copy of csrc/ in a temporary directory.
Such builds compute WRONG results by design: their mvm_version() says
"variant NAME" and they live only under lib/ab/.
"""
import os
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as G  # noqa: E402

args = sys.argv[1:]
name, patches, macros = args[0], [], []
i = 1
while i < len(args):
    if args[i] == "--patch":
        patches.append(args[i + 1])
        i += 2
    else:
        macros.append(args[i])
        i += 1
out_dir = os.path.join(G.LIB_DIR, "ab")
os.makedirs(out_dir, exist_ok=True)
out = os.path.join(out_dir, name + ".so")
with tempfile.TemporaryDirectory() as tmp:
    src = os.path.join(tmp, "bpc_baseline_amd", "csrc")
    shutil.copytree(os.path.join(G.PKG, "csrc"), src)
    for p in patches:
        with open(os.path.join(REPO, "tools", "diag", p + ".patch")) as fh:
            subprocess.run(["patch", "-s", "-p1"], cwd=tmp, stdin=fh, check=True)
    srcs = [os.path.join(src, os.path.basename(f)) for f in G.HIP_SRCS]
    variant = [f'-DMVM_VARIANT="{name}"'] if (patches or macros) else []
    subprocess.run([G._hipcc(), *G.HIPCC_FLAGS, "-I" + src, *variant, *("-D" + m for m in macros),
                    "-o", out, *srcs], check=True)
print(out)
