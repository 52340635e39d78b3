"""Performance experiment (not part of the product): lanes per wave of the straight-line
kernels (codegen.ALL_LANES). With 64 lanes a 64-instance block is one wave; with 32 or 16 it
is split over 2 or 4 partly filled waves, so a small batch spreads over more CUs (config 4's
4,096 instances are 64 full waves on 256 CUs).

  python tools/exp_lanes.py             # build tools/exp_lib/libmjhip_l{64,32,16}.so
  python tools/exp_lanes.py run         # GPU box: time config 4 (4,096) and the headline
                                        # (65,536) with each library, one process per library

Only the generated kernels' unit is rebuilt; the other units' objects come from build/obj.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tools", "exp_lib")
LANES = (64, 32, 16)


def build():
  import __graft_entry__ as ge
  from mujoco_inversedynamicstest_amd import codegen, models
  exp = os.path.join(ROOT, "tools", "exp", "lanes")
  os.makedirs(exp, exist_ok=True)
  for nl in LANES:
    saved = (codegen.ALL_LANES, dict(codegen.LANES))
    codegen.ALL_LANES = nl
    codegen.LANES = {st: nl for st in codegen.STAGES}
    try:
      entries = [(n, models.load(src, disable_contact=dc, disable_sensor=ds))
                 for n, src, dc, ds in ge.FAST_MODELS]
      inc = os.path.join(exp, f"gen_fast_l{nl}.inc")
      with open(inc, "w") as f:
        # the main unit only: the exact models' kernels stay in build/obj/gen_fast_exact.o
        f.write(codegen.generate_registries(entries)[0])
    finally:
      codegen.ALL_LANES, codegen.LANES = saved[0], saved[1]
    unit = os.path.join(exp, f"gen_fast_l{nl}.hip")
    src = open(os.path.join(ge.CSRC, "gen_fast.hip")).read()
    src = src.replace('#include "fast_kernels.h"', f'#include "{ge.CSRC}/fast_kernels.h"')
    src = src.replace('__has_include("gen_fast.inc")', "1").replace(
        '#include "gen_fast.inc"', f'#include "{inc}"')
    with open(unit, "w") as f:
      f.write(src)
    obj = os.path.join(exp, f"gen_fast_l{nl}.o")
    subprocess.run([os.environ.get("HIPCC", "/opt/rocm/bin/hipcc"), *ge.HIPCC_FLAGS,
                    "-I", ge.CSRC, "-c", "-o", obj, unit], check=True)
    objs = [os.path.join(ge.OBJ, u.replace(".hip", ".o")) for u in ge.UNITS
            if u != "gen_fast.hip"] + [obj]
    lib = os.path.join(OUT, f"libmjhip_l{nl}.so")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                    lib, *objs], check=True)
    print("built", lib)


def child(nl):
  import numpy as np
  from mujoco_inversedynamicstest_amd import engine, models
  from mujoco_inversedynamicstest_amd.sampler import sample_contact_states, sample_states
  engine.LIB_PATH = os.path.join(OUT, f"libmjhip_l{nl}.so")
  ref = None
  for name, contact, B in (("config 4", True, 4096), ("headline", False, 65536)):
    m = models.load("humanoid", disable_contact=not contact)
    q, v, a = sample_contact_states(m, B) if contact else sample_states(m, B)
    e = engine.InverseEngine(m, capacity=B, specialize=False)
    f = e.inverse(q, v, a)
    e.upload_states(q, v, a)
    t = min(e.time_kernel(B, 30) for _ in range(3))
    e.close()
    print(f"lanes {nl:2d} {name:9s} B={B:6d}: {t*1e3:8.1f} us per call "
          f"({B/t/1e3:.1f}M evals/s), qfrc sum {np.sum(f):.17g}", flush=True)
    ref = f


def run():
  for nl in LANES:
    r = subprocess.run([sys.executable, __file__, "child", str(nl)], capture_output=True,
                       text=True, timeout=240)
    print(r.stdout.strip())
    if r.returncode:
      print(r.stderr[-2000:])
      raise SystemExit(r.returncode)


if __name__ == "__main__":
  if len(sys.argv) > 2 and sys.argv[1] == "child":
    child(int(sys.argv[2]))
  elif len(sys.argv) > 1 and sys.argv[1] == "run":
    run()
  else:
    build()
