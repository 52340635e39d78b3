"""Performance experiment (not part of the product): where the generic pipeline spends time.

  python tools/exp_phases.py            # build tools/exp/libmjhip_phase.so (no GPU needed)
  python tools/exp_phases.py run [B]    # GPU box: config-4 humanoid (contacts on)

Builds libmjhip with -DMJH_PHASE_TIMING: lane 0 of every wave of k_inverse<0, CONTACT> adds
the wall clock (100 MHz) at the MJH_PHASE marks of engine_device.h. The mean over waves of
mark k minus mark k-1 is the mean wall time a wave spends in phase k.
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

EXP = os.path.join(ROOT, "tools", "exp")
LIB = os.path.join(EXP, "libmjhip_phase.so")
PHASES = ["kinematics", "comPos+camlight+tendon", "crb+factorM", "collision",
          "makeConstraint", "transmission+invVelocity", "discrete+invConstraint",
          "rne+assembly"]
MARKS = [0, 1, 2, 3, 4, 5, 7, 8, 9]   # mark 6 (after invPosition) folds into phase 6


def build():
  import __graft_entry__ as ge
  ge.generate_fast_kernels()
  os.makedirs(EXP, exist_ok=True)
  subprocess.run(["/opt/rocm/bin/hipcc", *ge.HIPCC_FLAGS, "-DMJH_PHASE_TIMING", "-o", LIB,
                  os.path.join(ge.CSRC, "mjhip.hip")], check=True)


def run(B=4096, reps=5):
  import numpy as np
  import torch
  from mujoco_inversedynamicstest_amd import engine, models
  from mujoco_inversedynamicstest_amd.sampler import sample_contact_states
  engine.LIB_PATH = LIB
  L = engine.lib()
  L.mjhip_phaseRead.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
  torch.cuda.set_device(0)
  m = models.load("humanoid", disable_contact=False)
  q, v, a = sample_contact_states(m, B)
  eng = engine.InverseEngine(m, capacity=B)
  eng.upload_states(q, v, a)
  acc = (ctypes.c_ulonglong * 32)()
  eng.inverse(B, mirror_input=True)
  L.mjhip_phaseRead(acc)
  waves = (B + 63) // 64
  tot = np.zeros(len(MARKS) - 1)
  for _ in range(reps):
    eng.inverse(B, mirror_input=True)
    torch.cuda.synchronize()
    assert L.mjhip_phaseRead(acc) == 0
    t = np.array([acc[k] for k in MARKS], dtype=np.float64) / waves
    tot += np.diff(t) / 100.0          # 100 MHz ticks -> us
  tot /= reps
  print(f"batch {B}, {waves} waves, mean per-wave phase time (us):")
  for name, x in zip(PHASES, tot):
    print(f"  {name:28s} {x:9.1f}")
  print(f"  {'total':28s} {tot.sum():9.1f}", flush=True)
  eng.close()


if __name__ == "__main__":
  if len(sys.argv) > 1 and sys.argv[1] == "run":
    run(int(sys.argv[2]) if len(sys.argv) > 2 else 4096)
  else:
    build()
