"""Performance experiment (not part of the product): where humanoid100's collision phase
spends its time. Each variant switches off the collisions of one class of geoms (contype =
conaffinity = 0, so the static collision program drops their pairs) and reads the per-stage
timers of one call of the generic kernel; the difference to the full model is what that
class of pairs costs (their narrowphase and their contacts' rows).

  python tools/exp_h100_collision.py [B]      # GPU box
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

PLANE, SPHERE, CAPSULE, ELLIPSOID, CYLINDER, BOX = 0, 2, 3, 4, 5, 6
VARIANTS = [
    ("all", ()),
    ("no ellipsoid/cylinder", (ELLIPSOID, CYLINDER)),
    ("no box", (BOX,)),
    ("no capsule", (CAPSULE,)),
    ("no sphere", (SPHERE,)),
    ("floor only for the 100", "free"),
    ("ellipsoid/cylinder half size", "shrink"),   # bounding spheres kept: GJK, little EPA
    ("ccd_iterations 10", "iters"),
]


def main():
  import numpy as np
  import torch
  from mujoco_inversedynamicstest_amd import engine, models
  import humanoid100_states as H
  B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
  torch.cuda.set_device(0)
  base = models.load("humanoid100")
  q, v, a = H.states(base, B, seed=1)
  only = os.environ.get("VARIANTS")
  for name, off in VARIANTS:
    if only and name not in only.split(","):
      continue
    m = models.load("humanoid100")
    t = np.asarray(m.geom_type)
    if off == "shrink":
      sel = (t == ELLIPSOID) | (t == CYLINDER)
      m.geom_size[sel] *= 0.5
    elif off == "iters":
      m.opt["ccd_iterations"] = 10
    elif off == "free":                       # the free primitives touch only the floor
      sel = np.asarray(m.geom_bodyid) >= m.nbody - 100     # the 100 free bodies come last
      m.geom_conaffinity[sel] = 0
      m.geom_contype[sel] = 2
      m.geom_conaffinity[t == PLANE] = 3
    else:
      for ty in off:
        m.geom_contype[t == ty] = 0
        m.geom_conaffinity[t == ty] = 0
    e = engine.InverseEngine(m, capacity=B, max_contacts=512, max_rows=1024)
    try:
      e.upload_states(q, v, a)
      e.inverse(B, mirror_input=True)
      torch.cuda.synchronize()
      e.timers(True)
      e.inverse(B, mirror_input=True)
      tm = e.timer_read()
      _, st = e.inverse(q, v, a, status=True)
      ncon = e.field_int("con_count", 0, min(B, 256))[:, 0].mean()
    finally:
      e.close()
    print(f"{name:26s} ncon {ncon:6.1f} flagged {int((st != 0).sum())}  " +
          ", ".join(f"{k} {x:.1f}" for k, (x, n) in tm.items()
                    if n and k in ("INVERSE", "POS_COLLISION", "POS_MAKE", "VELOCITY",
                                   "CONSTRAINT")), flush=True)


if __name__ == "__main__":
  main()
