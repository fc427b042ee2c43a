"""Build a variant libdx.so for same-box A/B runs (tools/ab_lib.sh):

  python tools/build_variant.py NAME [-DFOO=1 ...]

copies dexterity_amd/csrc to variants/NAME/csrc, builds it there with the extra flags
(and its own scene specializations) into variants/NAME/libdx.so.  Run the bench with
DX_LIB=variants/NAME/libdx.so."""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dexterity_amd import build as B  # noqa: E402

args = sys.argv[1:]
rev = None
if args and args[0].startswith("--rev="):  # the sources of a git revision instead of the tree
    rev = args.pop(0)[len("--rev="):]
name, extra = args[0], tuple(args[1:])
vdir = os.path.join(ROOT, "variants", name)
src = os.path.join(vdir, "csrc")
if os.path.exists(src):
    shutil.rmtree(src)
if rev:
    import subprocess

    os.makedirs(src)
    files = subprocess.run(["git", "-C", ROOT, "ls-tree", "--name-only", f"{rev}:dexterity_amd/csrc"],
                           check=True, capture_output=True, text=True).stdout.split()
    for f in files:
        data = subprocess.run(["git", "-C", ROOT, "show", f"{rev}:dexterity_amd/csrc/{f}"], check=True,
                              capture_output=True).stdout
        open(os.path.join(src, f), "wb").write(data)
else:
    shutil.copytree(B.CSRC, src)
# a revision from before the solver became a specialization dimension (round 5)
if "X(solver)" not in open(os.path.join(src, "dx_device.h")).read():
    B.DIMS = tuple(d for d in B.DIMS if d != "solver")
    B.SOLVER_SPECS = ()
# csrc includes "../../include/dx.h"
os.makedirs(os.path.join(ROOT, "variants", "include"), exist_ok=True)
shutil.copy(os.path.join(ROOT, "include", "dx.h"), os.path.join(ROOT, "variants", "include", "dx.h"))
B.CSRC = src
B.SPECS = os.path.join(src, "dx_specs.inc")
B.OUT = os.path.join(vdir, "libdx.so")
B.OBJ = os.path.join(vdir, "obj")
B.FLAGS = B.FLAGS + extra
print(B.build(force=True, verbose=False))
