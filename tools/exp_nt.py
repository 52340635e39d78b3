"""Performance experiment (not part of the product): the headline kernels without streaming
stores (codegen.NT_STORES compiled with -DMJHIP_NO_NT), for an A/B against the product build.

  python tools/exp_nt.py     # after __graft_entry__.build(): links build/obj/mjhip.o with a
                             # -DMJHIP_NO_NT gen_fast object into tools/exp_lib/libmjhip_nont.so
  MJHIP_LIB=tools/exp_lib/libmjhip_nont.so python bench.py ...   # on the GPU box
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

OUT = os.path.join(ROOT, "tools", "exp_lib", "libmjhip_nont.so")

if __name__ == "__main__":
  hipcc = "/opt/rocm/bin/hipcc"
  gen_o = os.path.join(ge.OBJ, "gen_fast_nont.o")
  subprocess.run([hipcc, *ge.HIPCC_FLAGS, "-DMJHIP_NO_NT", "-c", "-o", gen_o,
                  os.path.join(ge.CSRC, "gen_fast.hip")], check=True)
  os.makedirs(os.path.dirname(OUT), exist_ok=True)
  subprocess.run([hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", OUT,
                  os.path.join(ge.OBJ, "mjhip.o"), gen_o], check=True)
  print(OUT)
