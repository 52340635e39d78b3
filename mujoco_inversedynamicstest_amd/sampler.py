"""Counter-based synthetic state sampler.

Every instance i draws from its own stream u(i, k) = mix64(seed + GOLDEN*(i*STRIDE + k))
(splitmix64 finalizer), so a shard [first, first+n) produces exactly the rows the full
batch would: results are independent of the number of GPUs/ranks.

Per instance (humanoid, config 2):
  free joint position  U(-1,1) x U(-1,1) x U(0.8,1.4); quaternion = normalized N(0,1)^4
  limited hinge/slide  U(lo + margin*w, hi - margin*w)        (w = hi - lo)
  unlimited hinge      U(-pi, pi); unlimited slide U(-0.1, 0.1); ball = random unit quat
  qvel ~ N(0,1), qacc ~ N(0, acc_std), all fp64
With resample_tendons=True, instances whose fixed-tendon lengths fall outside a limited
tendon's range redraw all joint positions (next attempt of their stream) until none does,
which guarantees nefc = 0 when margin > 0 (no joint or tendon limit active).
"""
from __future__ import annotations

import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
STRIDE = 1 << 16       # draws per instance stream
ATTEMPT = 256          # draws reserved per resampling attempt
SEED = 20250314


def _mix64(z):
  z = z.copy()
  z ^= z >> np.uint64(30)
  z *= np.uint64(0xBF58476D1CE4E5B9)
  z ^= z >> np.uint64(27)
  z *= np.uint64(0x94D049BB133111EB)
  z ^= z >> np.uint64(31)
  return z


def _uniform(seed, idx, k):
  """U[0,1) doubles for instance indices idx (uint64 array) and draw numbers k (int array)."""
  with np.errstate(over="ignore"):
    ctr = idx * np.uint64(STRIDE) + np.asarray(k, dtype=np.uint64)
    z = _mix64(np.uint64(seed) + GOLDEN * ctr)
  return (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


class _Stream:
  def __init__(self, seed, idx, base):
    self.seed, self.idx, self.k = seed, idx, np.asarray(base, dtype=np.int64)

  def uniform(self, n):
    out = np.empty((len(self.idx), n))
    for j in range(n):
      out[:, j] = _uniform(self.seed, self.idx, self.k + j)
    self.k = self.k + n
    return out

  def normal(self, n):
    m = (n + 1) // 2
    u = self.uniform(2 * m)
    u1 = np.maximum(u[:, 0::2], 1e-300)
    u2 = u[:, 1::2]
    r = np.sqrt(-2.0 * np.log(u1))
    z = np.concatenate([r * np.cos(2 * np.pi * u2), r * np.sin(2 * np.pi * u2)], axis=1)
    return z[:, :n]


def _positions(m, st, margin):
  B = len(st.idx)
  q = np.tile(m.qpos0.astype(np.float64), (B, 1))
  for j in range(m.njnt):
    t = int(m.jnt_type[j])
    a = int(m.jnt_qposadr[j])
    if t == 0:
      u = st.uniform(3)
      q[:, a] = 2 * u[:, 0] - 1
      q[:, a + 1] = 2 * u[:, 1] - 1
      q[:, a + 2] = 0.8 + 0.6 * u[:, 2]
      g = st.normal(4)
      q[:, a + 3:a + 7] = g / np.linalg.norm(g, axis=1, keepdims=True)
    elif t == 1:
      g = st.normal(4)
      q[:, a:a + 4] = g / np.linalg.norm(g, axis=1, keepdims=True)
    else:
      u = st.uniform(1)[:, 0]
      if m.jnt_limited[j]:
        lo, hi = m.jnt_range[j]
        w = hi - lo
        lo2, hi2 = lo + margin * w, hi - margin * w
        q[:, a] = lo2 + (hi2 - lo2) * u
      elif t == 3:
        q[:, a] = -np.pi + 2 * np.pi * u
      else:
        q[:, a] = -0.1 + 0.2 * u
  return q


def _tendon_ok(m, q, tmargin):
  ok = np.ones(q.shape[0], dtype=bool)
  for t in range(m.ntendon):
    if not m.tendon_limited[t] or m.wrap_type[m.tendon_adr[t]] != 1:   # fixed tendons only
      continue
    L = np.zeros(q.shape[0])
    for w in range(m.tendon_adr[t], m.tendon_adr[t] + m.tendon_num[t]):
      L += m.wrap_prm[w] * q[:, m.jnt_qposadr[m.wrap_objid[w]]]
    lo, hi = m.tendon_range[t]
    ok &= (L - lo > tmargin) & (hi - L > tmargin)
  return ok


def sample_states(m, n, first=0, seed=SEED, margin=0.05, acc_std=10.0,
                  resample_tendons=True, max_attempts=200):
  """Return (qpos [n,nq], qvel [n,nv], qacc [n,nv]) for instances first..first+n-1."""
  idx = np.arange(first, first + n, dtype=np.uint64)
  st = _Stream(seed, idx, np.zeros(n, dtype=np.int64))
  qpos = _positions(m, st, margin)
  if resample_tendons and m.ntendon:
    tm = 1e-9
    bad = ~_tendon_ok(m, qpos, tm)
    attempt = 1
    while bad.any():
      if attempt >= max_attempts:
        raise RuntimeError("tendon-range resampling did not converge")
      sub = _Stream(seed, idx[bad], np.full(int(bad.sum()), attempt * ATTEMPT))
      qpos[bad] = _positions(m, sub, margin)
      bad_idx = np.nonzero(bad)[0]
      still = ~_tendon_ok(m, qpos[bad], tm)
      bad = np.zeros(n, dtype=bool)
      bad[bad_idx[still]] = True
      attempt += 1
  vst = _Stream(seed, idx, np.full(n, (max_attempts + 1) * ATTEMPT))
  qvel = vst.normal(m.nv)
  qacc = acc_std * vst.normal(m.nv)
  return qpos, qvel, qacc


def sample_contact_states(m, n, first=0, seed=SEED + 4, hinge_std=0.02, z_noise=0.02,
                          vel_std=0.5, acc_std=5.0):
  """Config 4: keyframe poses with noise, contacts on.

  Instance i takes keyframe i % nkey (squat, stand_on_left_leg, prone, supine for the
  humanoid), adds N(0, hinge_std) to every hinge/slide coordinate and U(-z_noise, z_noise)
  to the height of each free joint; qvel ~ N(0, vel_std), qacc ~ N(0, acc_std). Same
  counter-based streams as sample_states, so shards are world-size independent.
  """
  if not m.nkey:
    raise ValueError("model has no keyframes")
  idx = np.arange(first, first + n, dtype=np.uint64)
  st = _Stream(seed, idx, np.zeros(n, dtype=np.int64))
  key = (np.arange(first, first + n) % m.nkey).astype(np.int64)
  q = np.array(m.key_qpos, dtype=np.float64).reshape(m.nkey, m.nq)[key].copy()
  noise = st.normal(m.nq)
  zn = st.uniform(1)[:, 0] * 2 - 1
  for j in range(m.njnt):
    t = int(m.jnt_type[j])
    a = int(m.jnt_qposadr[j])
    if t in (2, 3):                       # slide, hinge
      q[:, a] += hinge_std * noise[:, a]
    elif t == 0:                          # free: height only
      q[:, a + 2] += z_noise * zn
  v = vel_std * st.normal(m.nv)
  acc = acc_std * st.normal(m.nv)
  return q, v, acc
