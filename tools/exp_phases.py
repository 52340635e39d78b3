"""Performance experiment (not part of the product): where the generic pipeline spends time.

  python tools/exp_phases.py            # build tools/exp/libmjhip_phase.so (no GPU needed)
  python tools/exp_phases.py run [B]    # GPU box: config-4 humanoid (contacts on)

Builds libmjhip with -DMJH_PHASE_TIMING (which adds per-contact spans to the product's
per-stage timer marks) and reads the raw mark sums of a timed context (mjhip_contextTimers):
lane 0 of every wave adds the wall clock (100 MHz) at the MJH_PHASE marks of engine_device.h.
The mean over waves of mark k minus mark k-1 is the mean wall time a wave spends in phase k.
"""
import ctypes
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

EXP = os.path.join(ROOT, "tools", "exp")
# PHASE_CQ=n builds/runs a variant with n lanes per contact in the cooperative contact rows
CQ = os.environ.get("PHASE_CQ", "")
LIB = os.path.join(ROOT, "tools", "exp_lib",
                   f"libmjhip_phase{'_cq' + CQ if CQ else ''}.so")   # travels to the GPU box
# generic pipeline (k_inverse): marks 0-9; constraint kernel after the generated kernels
# (k_constraint, mjh::constraintOnly): marks 10-13
GROUPS = [
    ("generic k_inverse", [0, 1, 2, 3, 4, 5, 7, 8, 9],   # mark 6 folds into phase 6
     ["kinematics", "comPos+camlight+tendon", "crb+factorM", "collision", "makeConstraint",
      "transmission+invVelocity", "discrete+invConstraint", "rne+assembly"]),
    ("k_constraint", [10, 11, 12, 13],
     ["collision", "makeConstraint", "reference+invConstraint"]),
    ("k_constraint_coop", [14, 15, 18, 16, 17],
     ["collision", "equality+friction+limit rows", "contact rows", "J'force+assembly"]),
]


def build():
  import __graft_entry__ as ge
  ge.generate_fast_kernels()
  # every unit with the spans compiled in (the generated kernels' object is kept between
  # builds: they carry the product's stage marks only)
  cq = [f"-DMJHIP_COOP_CQ={CQ}"] if CQ else []
  os.makedirs(os.path.dirname(LIB), exist_ok=True)
  ge.compile_library(LIB, os.path.join(EXP, f"obj{CQ}"), ["-DMJH_PHASE_TIMING", *cq],
                     reuse=("gen_fast.hip",))


def run(B=4096, reps=5):
  import numpy as np
  import torch
  from mujoco_inversedynamicstest_amd import engine, models
  from mujoco_inversedynamicstest_amd.sampler import sample_contact_states
  engine.LIB_PATH = LIB
  L = engine.lib()
  L.mjhip_phaseRead.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong)]
  torch.cuda.set_device(0)
  m = models.load("humanoid", disable_contact=False)
  q, v, a = sample_contact_states(m, B)
  eng = engine.InverseEngine(m, capacity=B)
  eng.upload_states(q, v, a)
  eng.timers(True)
  G = 16 if os.environ.get("MJHIP_COOP_LANES", "16") != "0" else 64
  acc = (ctypes.c_ulonglong * 48)()
  for generic in (False, True):
    eng.inverse(B, mirror_input=True, generic=generic)
    torch.cuda.synchronize()
    L.mjhip_phaseRead(eng.ctx, acc)
    waves = (B + 63) // 64
    sums = np.zeros(48)
    for _ in range(reps):
      t0 = time.perf_counter()
      eng.inverse(B, mirror_input=True, generic=generic)
      torch.cuda.synchronize()
      wall = time.perf_counter() - t0
      assert L.mjhip_phaseRead(eng.ctx, acc) == 0
      sums += np.array(acc[:48], dtype=np.float64)
    print(f"batch {B}, {waves} waves, {'generic' if generic else 'default'} dispatch "
          f"(last call {wall*1e3:.2f} ms wall); mean per-wave phase time (us):")
    for title, marks, names in GROUPS:
      # the cooperative kernel runs G lanes per instance: 64/G instances per wave
      nw = (B + 64 // G - 1) // (64 // G) if title == "k_constraint_coop" else waves
      t = sums[marks] / (reps * nw)
      if not t.any():
        continue
      d = np.diff(t) / 100.0           # 100 MHz ticks -> us
      print(f" {title}")
      for name, x in zip(names, d):
        print(f"  {name:28s} {x:9.1f}")
      print(f"  {'total':28s} {d.sum():9.1f}", flush=True)
    # spans inside one contact's rows (lane 0 of each wave): slot k sums, k + 1 counts
    spans = [("contact data+impedance", 40), ("contact dof loop", 42), ("contact finish", 44)]
    if sums[41] > 0:
      print(" per contact (lane 0's contacts, mean us)")
      for name, k in spans:
        print(f"  {name:28s} {sums[k] / sums[k + 1] / 100.0:9.2f}  ({int(sums[k + 1] / reps)} "
              f"contacts per call)")
  eng.close()


if __name__ == "__main__":
  if len(sys.argv) > 1 and sys.argv[1] == "run":
    run(int(sys.argv[2]) if len(sys.argv) > 2 else 4096)
  else:
    build()
