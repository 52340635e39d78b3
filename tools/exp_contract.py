"""Performance/parity experiment (not part of the product): the constraint kernels' unit
(kern_constraint.hip: the one-lane k_constraint that serves models with native-solver pairs,
and k_constraint_coop) compiled without multiply-add contraction, as the generic kernel's unit
is. The solver region of engine_device.h is contract(off) already, but the small helpers it
inlines (dot3, sub3, mulMatVec3, ...) are defined above that region and keep contraction.

  python tools/exp_contract.py      # build tools/exp_lib/libmjhip_ccoff.so (no GPU needed)
  MJHIP_LIB=tools/exp_lib/libmjhip_ccoff.so python -m pytest tests/test_convex_gpu.py -s ...
"""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
  import __graft_entry__ as ge
  out = os.path.join(ROOT, "tools", "exp_lib")
  objdir = os.path.join(ROOT, "tools", "exp", "ccoff_obj")
  os.makedirs(out, exist_ok=True)
  os.makedirs(objdir, exist_ok=True)
  for u in ge.UNITS:                       # every other unit's object as the product built it
    if u != "kern_constraint.hip":
      o = u.replace(".hip", ".o")
      shutil.copy2(os.path.join(ge.OBJ, o), os.path.join(objdir, o))
  ge.UNIT_FLAGS["kern_constraint.hip"] = ["-ffp-contract=off", "-DMJH_CONTRACT_OFF=1"]
  ge.compile_library(os.path.join(out, "libmjhip_ccoff.so"), objdir,
                     reuse=[u for u in ge.UNITS if u != "kern_constraint.hip"])
  print("built", os.path.join(out, "libmjhip_ccoff.so"))


if __name__ == "__main__":
  main()
