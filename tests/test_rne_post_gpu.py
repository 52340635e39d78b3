"""rne_post models on the MI355X: the device at the reference's static equilibria (and at
perturbed moving states around them) against the oracle to 1e-10, and its force/torque
readings against the values the reference's TestConnect / TestWeld expect
(engine_core_smooth_test.cc:165-303) to their 1e-6."""
import numpy as np
import pytest

from mujoco_inversedynamicstest_amd import engine
from oracle.oracle import Oracle

import rne_post_cases as rp
from test_gpu import assert_close

pytestmark = pytest.mark.gpu
CASES = rp.cases()


@pytest.mark.parametrize("name", sorted(CASES))
def test_rne_post_device(name):
  c = CASES[name]
  m = rp.load(name)
  o = Oracle(m)
  q0, _ = rp.equilibrium(m, o)
  B = 64
  rng = np.random.default_rng(11)
  q = np.stack([q0] + [rp.integrate_pos(m, q0, 0.05 * rng.standard_normal(m.nv))
                       for _ in range(B - 1)])
  v = np.vstack([np.zeros(m.nv), rng.standard_normal((B - 1, m.nv))])
  a = np.vstack([np.zeros(m.nv), rng.standard_normal((B - 1, m.nv))])
  e = engine.InverseEngine(m, capacity=B)
  f, st = e.inverse(q, v, a, status=True)
  assert (st == 0).all()
  sd = e.field("sensordata", 0, B)
  qc = e.field("qfrc_constraint", 0, B)
  counts = e.field_int("efc_count", 0, B)
  ref = {k: [] for k in ("qfrc_inverse", "qfrc_constraint", "sensordata")}
  for i in range(B):
    o.inverse(q[i], v[i], a[i])
    assert counts[i, 0] == o.efc.nefc and counts[i, 1] == o.efc.ne
    for k in ref:
      ref[k].append(getattr(o.d, k).copy())
  e.close()
  assert_close(f, np.array(ref["qfrc_inverse"]), "qfrc_inverse")
  assert_close(qc, np.array(ref["qfrc_constraint"]), "qfrc_constraint")
  assert_close(sd, np.array(ref["sensordata"]), "sensordata")
  for adr, expect in c["checks"]:
    np.testing.assert_allclose(sd[0, adr:adr + 3], expect, rtol=0, atol=1e-6,
                               err_msg=f"{name} device sensordata ({c['test']})")
