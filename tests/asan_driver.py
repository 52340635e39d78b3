"""Child process of tests/test_asan.py: exercises the sanitizer builds of the oracle
(ORACLE_LIB) and of the host-compiled device pipeline (KERNEL_HARNESS_FLAGS) on every code
path the CPU tests reach, and checks that both still agree bit for bit. Any invalid access
or undefined behaviour aborts the process (AddressSanitizer / -fno-sanitize-recover)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from kernel_harness import KernelCPU  # noqa: E402
from mujoco_inversedynamicstest_amd import models  # noqa: E402
from mujoco_inversedynamicstest_amd.sampler import sample_contact_states, sample_states  # noqa
from oracle.oracle import Oracle  # noqa: E402


def check(name, m, q, v, a, fd=False, caps=(None, None)):
  o, k = Oracle(m), KernelCPU(m, efc_cap=caps[0], con_cap=caps[1])
  for i in range(len(q)):
    ref = o.inverse(q[i], v[i], a[i])
    got, _ = k.inverse(q[i], v[i], a[i])
    if not np.array_equal(ref, got):
      raise SystemExit(f"{name}[{i}]: host device build differs from the oracle")
    k.inverse(q[i], v[i], a[i], classic=True)
    o.inverse(skipstage=2)            # mjSTAGE_VEL
    o.rne(1)
  if fd:
    o.set_state(q[0], v[0], a[0])
    o.inverse_fd(1e-6, dmdq=True, sensors=m.nsensor > 0)
  o.forward()
  o.compare_fwd_inv()
  print(f"{name}: {len(q)} states ok", flush=True)


def main():
  hc = models.load("humanoid")
  q, v, a = sample_contact_states(hc, 24)
  check("humanoid+contacts", hc, q, v, a)
  h = models.load("humanoid", disable_contact=True)
  q, v, a = sample_states(h, 16, margin=-0.1)        # limits active
  check("humanoid+limits", h, q, v, a, fd=True)
  for name in ("slider_crank", "inverse_test", "inertia", "linear", "weld", "connect",
               "equality_site", "equality_compare"):
    m = models.load(name)
    q, v, a = sample_states(m, 8, margin=-0.1)
    check(name, m, q, v, a, fd=name != "slider_crank")
  # round-2 paths: wrapping spatial tendons, site-relative and adhesion transmissions,
  # box-box contacts
  from mujoco_inversedynamicstest_amd import mjcf
  import test_tendon_cpu as T
  import test_transmission_cpu as R
  wm = mjcf.load_xml_string(T.WRAP)
  st = T._wrap_states(wm, 8, 3)
  check("wrap", wm, *(np.array([x[j] for x in st]) for j in range(3)))
  rm = mjcf.load_xml_string(R.REFSITE)
  rng = np.random.default_rng(2)
  check("refsite", rm, rng.uniform(-1, 1, (8, rm.nq)), rng.normal(size=(8, rm.nv)),
        rng.normal(size=(8, rm.nv)))
  am = R._adhesion("pyramidal", 3, 0.01, 0.005, 0.1)
  q = np.tile(am.qpos0, (8, 1))
  q[:, 2] = 0.1 + 0.02 * rng.normal(size=8)
  check("adhesion", am, q, rng.normal(size=(8, am.nv)), rng.normal(size=(8, am.nv)))
  bm = mjcf.load_xml_string("""<mujoco><worldbody>
    <body pos="0 0 .5"><freejoint/><geom type="box" size=".2 .15 .1"/></body>
    <body pos=".3 0 .5"><freejoint/><geom type="box" size=".1 .12 .08"/></body>
    </worldbody></mujoco>""")
  q = np.tile(bm.qpos0, (16, 1))
  for b in range(2):
    qq = rng.normal(size=(16, 4))
    q[:, 7 * b + 3:7 * b + 7] = qq / np.linalg.norm(qq, axis=1, keepdims=True)
  q[:, 7:10] = q[:, 0:3] + rng.uniform(-0.25, 0.25, (16, 3))
  check("boxbox", bm, q, rng.normal(size=(16, bm.nv)), rng.normal(size=(16, bm.nv)))
  # round 4: the 627-dof humanoid100 (attach/replicate) with ~150 contacts, capped context
  import humanoid100_states as H
  m = H.model()
  check("humanoid100", m, *H.states(m, 2, seed=9), caps=(H.MAX_ROWS, H.MAX_CONTACTS))
  print("ASAN_DRIVER_OK", flush=True)


if __name__ == "__main__":
  main()
