"""Per-stage timers (mjhip_contextTimers / mjhip_timerRead): the reference's mjTIMER_* table
(engine_inverse.c:38-67, :170-191, :199-260) for batched calls, on the GPU.

Checks: the slots the inverse path fills (INVERSE, POSITION and its four parts, VELOCITY,
CONSTRAINT) accumulate per call and count the calls; POSITION is the sum of its parts; each
stage's mean wave time is below the call's wall time; timing changes no result bit; reset
clears; timers off leave the table alone. Straight-line path with the cooperative constraint
kernel (humanoid with contacts), the one-lane constraint kernel (slider-crank) and the generic
kernel.
"""
import numpy as np
import pytest

from mujoco_inversedynamicstest_amd import engine, models
from mujoco_inversedynamicstest_amd.sampler import sample_contact_states, sample_states

pytestmark = pytest.mark.gpu

PARTS = ("POS_KINEMATICS", "POS_INERTIA", "POS_COLLISION", "POS_MAKE")


def _check(t, calls, collision, overlap=False):
  assert t["INVERSE"][1] == calls and t["INVERSE"][0] > 0
  for k in ("POSITION", "VELOCITY", "CONSTRAINT") + PARTS:
    assert t[k][1] == calls, k
  assert t["POSITION"][0] == pytest.approx(sum(t[k][0] for k in PARTS), rel=1e-12)
  assert t["POS_KINEMATICS"][0] > 0 and t["VELOCITY"][0] > 0 and t["CONSTRAINT"][0] > 0
  if collision:
    assert t["POS_COLLISION"][0] > 0 and t["POS_MAKE"][0] > 0
  if overlap:   # split launch (path 3): the constraint kernel runs beside the fac / va stages
    smooth = t["POS_KINEMATICS"][0] + t["POS_INERTIA"][0] + t["VELOCITY"][0]
    rows = t["POS_COLLISION"][0] + t["POS_MAKE"][0] + t["CONSTRAINT"][0]
    assert smooth <= t["INVERSE"][0] * 1.05 and rows <= t["INVERSE"][0] * 1.05
  else:
    stages = t["POSITION"][0] + t["VELOCITY"][0] + t["CONSTRAINT"][0]
    assert stages <= t["INVERSE"][0] * 1.05
  for k in ("STEP", "FORWARD", "ACTUATION", "ADVANCE", "POS_PROJECT", "COL_BROAD",
            "COL_NARROW"):
    assert t[k] == (0.0, 0), k


@pytest.mark.parametrize("case", ["humanoid_contacts", "slider_crank", "generic"])
def test_timers(case):
  if case == "slider_crank":
    m = models.load("slider_crank")
    rng = np.random.default_rng(3)
    B = 2048
    q, v, a = (rng.uniform(-np.pi, np.pi, (B, 3)), rng.normal(size=(B, 3)),
               rng.normal(size=(B, 3)))
  else:
    m = models.load("humanoid")
    B = 4096
    q, v, a = sample_contact_states(m, B)
  generic = case == "generic"
  e = engine.InverseEngine(m, capacity=B)
  try:
    f0 = e.inverse(q, v, a, generic=generic)
    e.timers(True)
    for _ in range(3):
      f1 = e.inverse(q, v, a, generic=generic)
      np.testing.assert_array_equal(f1, f0)
    t = e.timer_read()
    print(case, {k: (round(x, 4), n) for k, (x, n) in t.items() if n})
    _check(t, 3, collision=True, overlap=e.last_path == 3)
    t2 = e.timer_read(reset=True)
    assert t2 == t
    assert all(x == (0.0, 0) for x in e.timer_read().values())
    e.timers(False)
    e.inverse(q, v, a, generic=generic)
    assert all(x == (0.0, 0) for x in e.timer_read().values())
  finally:
    e.close()


def test_timers_no_contacts():
  """The headline configuration (contacts disabled, no constraint rows): the straight-line
  kernel's position and velocity stages."""
  m = models.load("humanoid", disable_contact=True)
  B = 65536
  q, v, a = sample_states(m, B)
  e = engine.InverseEngine(m, capacity=B)
  try:
    e.timers(True)
    e.inverse(q, v, a)
    t = e.timer_read()
    print({k: (round(x, 4), n) for k, (x, n) in t.items() if n})
    assert t["INVERSE"][1] == 1 and t["POS_KINEMATICS"][0] > 0 and t["VELOCITY"][0] > 0
    assert t["POS_INERTIA"][0] > 0 and t["POS_COLLISION"][0] == 0
  finally:
    e.close()


def test_timed_context_freed_then_another():
  """A timed context freed while timing is on detaches every unit's timer pointer before its
  stream and accumulator go: a second context then runs with identical results,
  may enable timers itself, and counts only its own calls."""
  m = models.load("humanoid")
  B = 1024
  q, v, a = sample_contact_states(m, B)
  e1 = engine.InverseEngine(m, capacity=B)
  f0 = e1.inverse(q, v, a)
  e1.timers(True)
  e1.inverse(q, v, a)
  e1.close()                               # freed with timers on
  e2 = engine.InverseEngine(m, capacity=B)
  try:
    np.testing.assert_array_equal(e2.inverse(q, v, a), f0)
    assert all(x == (0.0, 0) for x in e2.timer_read().values())
    e2.timers(True)                        # the freed context no longer holds the slot
    np.testing.assert_array_equal(e2.inverse(q, v, a), f0)
    _check(e2.timer_read(), 1, collision=True, overlap=e2.last_path == 3)
  finally:
    e2.close()
