"""Diagnostic: mjd_inverseFD stage-skip layouts (2: k_accskip + k_vaskip, 1: k_vaskip for both,
NOSKIP: the full pipeline) against each other, per output and perturbation, bit for bit."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from mujoco_inversedynamicstest_amd import engine, models
from mujoco_inversedynamicstest_amd.sampler import sample_states

name = sys.argv[1] if len(sys.argv) > 1 else "humanoid"
m = models.load(name, disable_contact=True)
for NB in (64, 1024):
  q, v, a = sample_states(m, NB, first=300)
  e = engine.InverseEngine(m, capacity=NB * (3 * m.nv + 1))
  res = {}
  for lay, env in (("2", {}), ("1", {"MJHIP_FD_NOACCSKIP": "1"}), ("full", {"MJHIP_FD_NOSKIP": "1"})):
    for k in ("MJHIP_FD_NOACCSKIP", "MJHIP_FD_NOSKIP"):
      os.environ.pop(k, None)
    os.environ.update(env)
    res[lay] = e.inverse_fd(q, v, a, eps=1e-6, dmdq=True)
  e.close()
  for lay in ("2", "1"):
    for nm, x, r in zip(("DfDq", "DfDv", "DfDa", "DmDq"), res[lay], res["full"]):
      bad = x != r
      print(f"NB={NB} layout {lay} {nm}: {bad.any(axis=(1, 2)).sum()}/{NB} bases differ,"
            f" {bad.sum()} elements; rows (perturbed dof) hit: {np.flatnonzero(bad.any(axis=(0, 2))).tolist()}"
            f" max abs {np.abs(x - r).max():.3e}")
