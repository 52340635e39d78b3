"""Predefined <contact><pair> elements on the GPU: the generic kernel and
the run-time specialized straight-line kernel with the cooperative constraint kernel (whose
host-built pair program merges the predefined pairs, csrc/mjhip.hip collision_pairs) against
the oracle's serial mj_collision merge (tests/test_pairs_cpu.py pins it).

Bar: the contacts exactly (count, geom pairs, dims, order), qfrc_inverse and the constraint
forces to the north-star 1e-10 normwise (the straight-line kernels contract multiply-adds)."""
import numpy as np
import pytest

from mujoco_inversedynamicstest_amd import engine
from oracle.oracle import Oracle

import pair_models as P

pytestmark = pytest.mark.gpu

RTOL = 1e-10


@pytest.mark.parametrize("specialize", [False, True])
def test_pairs_vs_oracle(specialize):
  m = P.mixed()
  B = 1000
  q, v, a = P.mixed_states(m, B, seed=21)
  e = engine.InverseEngine(m, capacity=B, specialize=specialize)
  try:
    assert (e.fast_kernel is not None) == specialize
    f, st = e.inverse(q, v, a, status=True)
    ncon = e.field_int("con_count", 0, B)[:, 0]
    cgeom = e.field_int("con_geom", 0, B)
    cdim = e.field_int("con_dim", 0, B)
    qc = e.field("qfrc_constraint", 0, B)
  finally:
    e.close()
  assert (st == 0).all()
  o = Oracle(m)
  err, total = 0.0, 0
  for i in range(B):
    ref = o.inverse(q[i], v[i], a[i])
    n = o.efc.ncon
    assert ncon[i] == n
    np.testing.assert_array_equal(cgeom[i, :2 * n], o.contact_field("con_geom").reshape(-1))
    np.testing.assert_array_equal(cdim[i, :n], o.contact_field("con_dim"))
    for mine, theirs in ((f[i], ref), (qc[i], o.d.qfrc_constraint)):
      err = max(err, np.abs(mine - theirs).max() / max(1.0, np.abs(theirs).max()))
    total += n
  print(f"specialize={specialize}: {total} contacts over {B} states, max error {err:.2e}")
  assert total > 2 * B
  assert err <= RTOL


def test_all_collisions_known_answer_gpu():
  """engine_collision_driver_test.cc:52-67 on the device: box/sphere_collides and
  box/sphere_predefined."""
  m = P.collisions()
  e = engine.InverseEngine(m, capacity=64, specialize=False)
  try:
    z = np.zeros((1, m.nv))
    e.inverse(m.qpos0[None], z, z)
    n = int(e.field_int("con_count", 0, 1)[0, 0])
    geoms = e.field_int("con_geom", 0, 1)[0, :2 * n].reshape(n, 2)
  finally:
    e.close()
  names = m.names["geom"]
  assert sorted(tuple(sorted((names[x], names[y]))) for x, y in geoms) == [
      ("box", "sphere_collides"), ("box", "sphere_predefined")]
