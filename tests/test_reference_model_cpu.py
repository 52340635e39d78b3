"""The reference's own inverse tests on their own model (engine_inverse_test.cc:32-123), CPU side.

test/testdata/model.xml (fixture tests/golden/testdata_model.npz) has everything the path
touches at once: a free base with hinge, ball and wheel legs, the icosahedron mesh on a
slider/hinge, the height field, a welded wrapping cylinder, free boxes, the fluid (both
models), gravity compensation, spatial and fixed tendons, ten actuators (dynamics incl.
integrator, filter, filterexact, intvelocity) and eleven sensors.

ForwardInverseMatch runs mj_step 70 times and checks mj_compareFwdInv's solver_fwdinv < 1e-10.
DiscreteInverseMatch finite-differences qvel over one step for Euler, implicit and
implicitfast and checks solver_fwdinv < 1e-9 with mjENBL_INVDISCRETE and > 1 without. The
forward constraint solver is outside this path, so both are restated in the form of
tests/test_oracle_pins.py:test_compare_fwd_inv_constrained: the forward solution is the
state's qacc, the applied forces are those that make it so (qfrc_applied = qfrc_inverse -
qfrc_actuator - J'xfrc), and the integrators' step maps it to the discrete acceleration
a' = H^-1 M a with H = M + h diag(damping) (Euler), M - h qDeriv (implicit, mjd_smooth_vel
with the bias and fluid terms) or M - h qDeriv reduced to qM's sparsity (implicitfast).
States: the model's keyframe (a state of the reference's own simulation), the free boxes on
the mesh and the height field, and perturbations (tests/reference_model_states.py).
"""
import numpy as np
import pytest

from kernel_harness import KernelCPU
from oracle.oracle import Oracle

import reference_model_states as R

mjENBL_INVDISCRETE = 1 << 3
INTEGRATORS = {"Euler": 0, "implicit": 2, "implicitfast": 3}


def _controls(m, rng):
  return rng.uniform(-1, 1, m.nu)


def test_forward_inverse_match():
  """solver_fwdinv of the constructed forward solution < 1e-10 (relative to the forces) on
  every state, with contact, limit and equality rows present."""
  m = R.model()
  q, v, a = R.states(m, 24, seed=1)
  o = Oracle(m)
  rng = np.random.default_rng(2)
  rows = 0
  for i in range(len(q)):
    o.d.ctrl[:] = _controls(m, rng)
    o.d.xfrc_applied[:] = 0.8 * (rng.random(6 * m.nbody) - 0.5)
    f = o.inverse(q[i], v[i], a[i])
    assert o.d.status == 0
    jx = np.zeros(m.nv)
    o.xfrc_accumulate(jx)
    o.d.qfrc_applied[:] = f - o.d.qfrc_actuator - jx
    rows += o.efc.nefc
    fw = o.compare_fwd_inv()
    assert o.efc.nefc > 0
    assert fw.max() < 1e-10 * max(1.0, np.abs(f).max()), (i, fw)
  assert rows > 24 * 5


def _discrete_acc(o, m, integ, a):
  """The acceleration the integrator's step realizes for the continuous solution a."""
  h = m.opt["timestep"]
  M = o.fullM()
  if integ == "Euler":
    H = M + h * np.diag(m.dof_damping)
  elif integ == "implicit":
    H = M - h * o.smooth_vel(1)
  else:
    # qDeriv reduced to qM's sparsity, applied through mj_mulM, which skips the off-diagonal
    # entries of "simple" dofs (dof_simplenum, engine_support.c mj_mulM): the coupling the
    # fluid adds between a free box's six dofs is dropped for those rows, as in the reference
    qd = o.smooth_vel(0)
    Dr = np.zeros_like(qd)
    for r in range(m.nv):
      Dr[r, r] = qd[r, r]
      c = m.dof_parentid[r]
      while c >= 0 and not m.dof_simplenum[r]:
        Dr[r, c] = Dr[c, r] = qd[r, c]
        c = m.dof_parentid[c]
    H = M - h * Dr
  return np.linalg.solve(H, M @ a)


@pytest.mark.parametrize("integ", list(INTEGRATORS))
def test_discrete_inverse_match(integ):
  """Discrete inverse dynamics of a' returns the continuous forces of a (< 1e-9 relative)
  with mjENBL_INVDISCRETE, and does not without it."""
  m, md = R.model(), R.model()
  m.opt["integrator"] = md.opt["integrator"] = INTEGRATORS[integ]
  md.opt["enableflags"] |= mjENBL_INVDISCRETE
  q, v, a = R.states(m, 12, seed=3)
  oc, od = Oracle(m), Oracle(md)
  rng = np.random.default_rng(4)
  for i in range(len(q)):
    ctrl = _controls(m, rng)
    oc.d.ctrl[:] = od.d.ctrl[:] = ctrl
    f_cont = oc.inverse(q[i], v[i], a[i])
    a_disc = _discrete_acc(oc, m, integ, a[i])
    f_disc = od.inverse(q[i], v[i], a_disc)
    assert od.d.status == 0
    np.testing.assert_array_equal(od.d.qacc, a_disc)
    scale = max(1.0, np.abs(f_cont).max())
    assert np.abs(f_disc - f_cont).max() <= 1e-9 * scale, np.abs(f_disc - f_cont).max()
    # without the flag: off by h-sized terms, three orders above the flag's bound
    assert np.abs(oc.inverse(q[i], v[i], a_disc) - f_cont).max() > 1e-6 * scale


@pytest.mark.parametrize("integ", list(INTEGRATORS))
def test_device_code_bitexact_invdiscrete(integ):
  """The device pipeline compiled for the host equals the oracle bit for bit under
  mjENBL_INVDISCRETE (fluid derivatives included for implicit and implicitfast)."""
  m = R.model()
  m.opt["integrator"] = INTEGRATORS[integ]
  m.opt["enableflags"] |= mjENBL_INVDISCRETE
  q, v, a = R.states(m, 9, seed=5)
  o, k = Oracle(m), KernelCPU(m)
  rng = np.random.default_rng(6)
  for i in range(len(q)):
    o.d.ctrl[:] = k.d.ctrl[:] = _controls(m, rng)
    f = o.inverse(q[i], v[i], a[i])
    g, st = k.inverse(q[i], v[i], a[i])
    assert st == o.d.status == 0
    np.testing.assert_array_equal(g, f)
    np.testing.assert_array_equal(k.d.qacc, o.d.qacc)
