"""Sparse-Jacobian models on the GPU: the reference's compressed rows
(mj_isSparse, engine_core_constraint.c:99-106) built by the generic kernel -- the 63-dof pile
(jacobian "auto", nv >= 60), a 27-dof pile with jacobian="sparse", and a model with every
row type (tests/sparse_models.py) -- against the oracle, which restates the sparse path:
counts, the compressed structure (nJ, rownnz, rowadr, colind of efc_J and efc_JT, the
tendon rows') exact; qfrc_inverse, efc_J/efc_JT values and the constraint forces to the
north-star 1e-10 (the generic kernel rounds as the oracle, so they are expected equal)."""
import numpy as np
import pytest

from mujoco_inversedynamicstest_amd import engine
from oracle.oracle import Oracle

import sparse_models as S

pytestmark = pytest.mark.gpu

RTOL = 1e-10


def _case(case):
  if case == "nv63_auto":
    m = S.pile()
    return m, S.states(m, 512, seed=7)
  if case == "nv27_sparse":
    m = S.pile(nfree=4, jacobian="sparse")
    return m, S.states(m, 512, seed=7)
  m = S.misc()
  return m, S.misc_states(m, 512, seed=7)


@pytest.mark.parametrize("case", ["nv63_auto", "nv27_sparse", "misc"])
def test_sparse_model_vs_oracle(case):
  m, (q, v, a) = _case(case)
  B = len(q)
  e = engine.InverseEngine(m, capacity=B)
  try:
    assert e.fast_kernel is None                  # compressed rows: the generic kernel
    f, st = e.inverse(q, v, a, status=True)
    nefc = e.field_int("efc_count", 0, B)[:, 0]
    nJ = e.field_int("nJ", 0, B)[:, 0]
    force = e.field("efc_force", 0, B)
    J, JT = e.field("efc_J", 0, B), e.field("efc_JT", 0, B)
    ints = {n: e.field_int(n, 0, B) for n in ("efc_J_rownnz", "efc_J_rowadr", "efc_J_colind",
                                             "efc_JT_rownnz", "efc_JT_rowadr",
                                             "efc_JT_colind", "ten_J_rownnz", "ten_J_colind")}
    tenv = e.field("ten_velocity", 0, B)
  finally:
    e.close()
  o = Oracle(m)
  err, rows, exact = 0.0, 0, 0
  for i in range(B):
    ref = o.inverse(q[i], v[i], a[i])
    assert st[i] == o.d.status == 0
    assert nefc[i] == o.efc.nefc and nJ[i] == o.efc.nJ
    sp = o.efc_sparse()
    n, k = o.efc.nefc, o.efc.nJ
    for name in ("efc_J_rownnz", "efc_J_rowadr"):
      np.testing.assert_array_equal(ints[name][i, :n], sp[name])
    for name in ("efc_J_colind", "efc_JT_colind"):
      np.testing.assert_array_equal(ints[name][i, :k], sp[name])
    if n:
      for name in ("efc_JT_rownnz", "efc_JT_rowadr"):
        np.testing.assert_array_equal(ints[name][i, :m.nv], sp[name])
    nt = m.sizes["ntendon"]
    tn = o.d.sparse("ten_J_rownnz")[:nt]
    np.testing.assert_array_equal(ints["ten_J_rownnz"][i, :nt], tn)
    np.testing.assert_array_equal(ints["ten_J_colind"][i, :tn.sum()],
                                  o.d.sparse("ten_J_colind")[:tn.sum()])
    scale = max(1.0, np.abs(ref).max())
    err = max(err, np.abs(f[i] - ref).max() / scale)
    for mine, theirs in ((J[i, :k], sp["efc_J"]), (JT[i, :k], sp["efc_JT"]),
                         (force[i, :n], o.efc_field("efc_force")), (tenv[i], o.d.ten_velocity)):
      if len(theirs):
        err = max(err, np.abs(mine - theirs).max() / max(1.0, np.abs(theirs).max()))
    exact += np.array_equal(f[i], ref)
    rows += n
  print(f"{case}: {rows} rows, max error {err:.2e}, qfrc_inverse bit-identical in "
        f"{exact}/{B}")
  assert rows > 10 * B
  assert err <= RTOL
