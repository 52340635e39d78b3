"""Multi-rank plumbing on CPU (gloo, world size 2): sharding is exact and independent of
the world size, and the rank-0 gather returns every rank's rows. Compute per rank uses the
oracle (CPU tests have no GPU); the GPU path shares the same shard/gather code (bench.py).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mujoco_inversedynamicstest_amd import models, parallel
from mujoco_inversedynamicstest_amd.sampler import sample_states


def test_shard_partition():
  for total in (0, 1, 63, 65536, 262144, 100001):
    for world in (1, 2, 3, 8):
      ranges = [parallel.shard(total, world, r) for r in range(world)]
      assert sum(c for _, c in ranges) == total
      pos = 0
      for first, count in ranges:
        assert first == pos
        pos += count


def test_sampler_shards_independent_of_world(humanoid):
  q, v, a = sample_states(humanoid, 1000)
  for world in (2, 8):
    parts = [sample_states(humanoid, c, first=f) for f, c in
             (parallel.shard(1000, world, r) for r in range(world))]
    np.testing.assert_array_equal(np.vstack([p[0] for p in parts]), q)
    np.testing.assert_array_equal(np.vstack([p[2] for p in parts]), a)


def _free_port():
  s = socket.socket()
  s.bind(("127.0.0.1", 0))
  port = s.getsockname()[1]
  s.close()
  return port


def _worker(rank, world, port, total, q):
  os.environ["MASTER_ADDR"] = "127.0.0.1"
  os.environ["MASTER_PORT"] = str(port)
  dist.init_process_group("gloo", rank=rank, world_size=world)
  from oracle.oracle import Oracle
  m = models.load("humanoid", disable_contact=True)
  first, count = parallel.shard(total, world, rank)
  qp, qv, qa = sample_states(m, count, first=first)
  o = Oracle(m)
  out = torch.tensor(np.array([o.inverse(qp[i], qv[i], qa[i]) for i in range(count)]))
  got = parallel.gather_to_rank0(out, world, rank, parallel.shard_counts(total, world))
  if rank == 0:
    q.put(torch.cat(got).numpy())
  dist.barrier()
  dist.destroy_process_group()


@pytest.mark.parametrize("total", [64, 65])
def test_gloo_world2_gather_matches_single_process(humanoid, total):
  """Even shards (64 over 2) and uneven ones (65: rank 0 holds 33 rows, rank 1 32), the
  receive sizes then coming from shard_counts as bench.py's --global-batch passes them."""
  world = 2
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  port = _free_port()
  procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
  for p in procs:
    p.start()
  res = q.get(timeout=240)
  for p in procs:
    p.join(timeout=120)
    assert p.exitcode == 0
  from oracle.oracle import Oracle
  qp, qv, qa = sample_states(humanoid, total)
  o = Oracle(humanoid)
  ref = np.array([o.inverse(qp[i], qv[i], qa[i]) for i in range(total)])
  np.testing.assert_array_equal(res, ref)
