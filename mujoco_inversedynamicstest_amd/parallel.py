"""Batch sharding over ranks (one process per GPU) and the RCCL gather to rank 0.

mj_inverse has no inter-instance dependence, so a global batch splits into
contiguous index shards with no data-path collective; states come from the counter-based
sampler, so a shard's rows are identical for any world size. The only collective is the
gather of results to rank 0 (north star: RCCL over xGMI, used only for that).
"""
from __future__ import annotations


def shard(total: int, world: int, rank: int):
  """Contiguous shard [first, first+count) of `total` instances for `rank` of `world`."""
  base, rem = divmod(total, world)
  first = rank * base + min(rank, rem)
  return first, base + (1 if rank < rem else 0)


def shard_counts(total: int, world: int):
  """Rows of every rank's shard (what rank 0 receives from each peer)."""
  return [shard(total, world, r)[1] for r in range(world)]


def gather_to_rank0(tensor, world: int, rank: int, counts=None):
  """Gather every rank's tensor to rank 0 (RCCL on GPU tensors, gloo on CPU tensors).

  Returns the list of gathered tensors on rank 0 (rank order) and None elsewhere. Uses
  point-to-point sends into rank 0 (RCCL has no native gather; each peer uses its own xGMI
  link). `counts` gives the leading dimension of each rank's tensor when shards are uneven
  (shard_counts); by default every rank's tensor has this rank's shape.
  """
  import torch
  import torch.distributed as dist
  if world == 1:
    return [tensor]
  if rank == 0:
    shape = list(tensor.shape)
    bufs = [tensor]
    for r in range(1, world):
      if counts is not None:
        shape[0] = counts[r]
      bufs.append(torch.empty(shape, dtype=tensor.dtype, device=tensor.device))
    ops = [dist.P2POp(dist.irecv, bufs[r], r) for r in range(1, world) if bufs[r].numel()]
    for req in (dist.batch_isend_irecv(ops) if ops else []):
      req.wait()
    return bufs
  if tensor.numel():
    for r in dist.batch_isend_irecv([dist.P2POp(dist.isend, tensor, 0)]):
      r.wait()
  return None
