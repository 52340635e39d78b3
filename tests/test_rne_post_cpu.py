"""The reference-held numbers on the inverse path: force/torque sensors of the rne_post
models at static equilibrium (TestConnect / TestWeld, engine_core_smooth_test.cc:165-303;
fixtures in tests/golden, equilibria by tests/rne_post_cases.py).

Each model's expected readings are the sensors' `user` attributes, written by the
reference's authors: -gravity times the mass the sensor's body carries through the connect
or weld (both bodies), and the matching torque. They exercise mj_inverse with equality rows
(connect, weld with torquescale 1 and 0, a joint equality and dof friction loss as
distractors), the impedance/reference/update of those rows, mj_rnePostConstraint's
equality branch (cfrc_ext from efc_force) and the force/torque sensors, in rotated frames.
The oracle must reproduce them to the reference's 1e-6; the device pipeline compiled for
the host must equal the oracle bit for bit at those states.
"""
import numpy as np
import pytest

from oracle.oracle import Oracle

import rne_post_cases as rp
from kernel_harness import KernelCPU

CASES = rp.cases()


def test_all_fixtures_present():
  assert len(CASES) == 15
  assert sum(c["test"] is not None for c in CASES.values()) == 14


@pytest.mark.parametrize("name", sorted(CASES))
def test_rne_post_sensor_readings(name):
  c = CASES[name]
  m = rp.load(name)
  o = Oracle(m)
  q, r = rp.equilibrium(m, o)
  floss = np.asarray(m.dof_frictionloss)
  held = floss == 0
  # at rest on every dof the equality rows hold; friction-loss dofs carry at most the loss
  assert np.abs(r[held]).max() <= 1e-9, r
  assert (np.abs(r[~held]) <= floss[~held]).all(), (r, floss)
  assert o.efc.ncon == 0 and o.efc.ne > 0
  for adr, expect in c["checks"]:
    np.testing.assert_allclose(o.d.sensordata[adr:adr + 3], expect, rtol=0, atol=1e-6,
                               err_msg=f"{name} sensordata[{adr}:{adr + 3}] ({c['test']})")


@pytest.mark.parametrize("name", sorted(CASES))
def test_rne_post_device_bitexact(name):
  """The device pipeline (host build) at the equilibrium and at perturbed moving states."""
  m = rp.load(name)
  o = Oracle(m)
  q0, _ = rp.equilibrium(m, o)
  rng = np.random.default_rng(7)
  states = [(q0, np.zeros(m.nv), np.zeros(m.nv))]
  for _ in range(3):
    states.append((rp.integrate_pos(m, q0, 0.05 * rng.standard_normal(m.nv)),
                   rng.standard_normal(m.nv), rng.standard_normal(m.nv)))
  k = KernelCPU(m, o.efc.capacity)
  for cl in (False, True):
    for q, v, a in states:
      o.inverse(q, v, a)
      _, st = k.inverse(q, v, a, classic=cl)
      assert st == 0 and k.d.nefc == o.d.nefc
      for f in ("qfrc_inverse", "qfrc_constraint", "sensordata", "cfrc_int", "cfrc_ext",
                "cacc"):
        np.testing.assert_array_equal(getattr(k.d, f), getattr(o.d, f), err_msg=f)
