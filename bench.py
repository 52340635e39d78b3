"""bench.py — mj_inverse evals/s, humanoid 27-DoF, batch 65,536 per GPU (BASELINE.json).

A step is one pass of the fused HIP mj_inverse over one batch of 65,536 synthetic humanoid
states (config-2 sampler, contacts disabled, every limit inactive) whose inputs are already
resident in the device mirror (HBM); every mjData output field of mj_inverse is written
(2,563 doubles per instance). With N GPUs each rank owns a contiguous shard of the global
batch and there is no collective in the timed region. After that region, rank 0 gathers
every rank's full qfrc_inverse (B x nv fp64) over RCCL point-to-point, and a second timed
region runs step + gather back to back, so scaling is reported with and without the gather
(SURVEY.md §8e).

  python bench.py [--gpus N] [--steps K] [--warmup W]      # spawns N ranks itself
  python bench.py --gpus 8 --global-batch 262144           # config 3 (32,768 per GPU)
  torchrun --nproc-per-node N bench.py --gpus N ...        # what the driver runs

Default per-GPU batch is 65,536 (weak scaling); --global-batch fixes the total instead
(strong scaling). Prints ONE JSON line on rank 0 (contract in the task statement).
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "mj_inverse evals/sec, humanoid 27-DoF, batch=65536 @ 1/2/4/8 MI355X vs host CPU"
HBM_PEAK_GBPS = 8000.0          # MI355X_MICROARCH.md chip table (spec)


def available_cores() -> int:
  """Host cores this process may run on: the affinity mask, capped by a cgroup-v2 CPU quota
  (a container's cpu.max) when one is set."""
  n = len(os.sched_getaffinity(0))
  try:
    quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
    if quota != "max":
      n = min(n, max(1, int(quota) // int(period)))
  except (OSError, ValueError):
    pass
  return n


def spawn_ranks(gpus: int) -> int:
  """Relaunch this script as `gpus` ranks (one process per GPU, torch.distributed.run on
  127.0.0.1) and return their exit code. Called before anything touches the GPU: the parent
  only waits for its child."""
  import socket
  with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
  cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
         f"--nproc-per-node={gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
         os.path.abspath(__file__)] + sys.argv[1:]
  return subprocess.call(cmd)


def pmc_traffic(eng, m, model, count, name="pmc_traffic.json"):
  """HBM bytes per launch from the newest committed PMC summary (tools/pmc.sh +
  tools/pmc_summary.py) whose kernels were built from the same generated source as the one
  this run launches (matched by codegen.source_hash, not by name), else None. Config 4's
  summary (pmc_traffic_c4.json) is per eval at its own batch and row counts."""
  import glob
  from mujoco_inversedynamicstest_amd import codegen
  if not eng.fast_kernel:
    return None, None
  sha = codegen.source_hash(m, eng.fast_kernel)
  for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", name)), reverse=True):
    rec = json.load(open(path))
    if rec.get("model") == model and rec.get("source_sha") == sha:
      per_eval = rec["traffic_bytes_per_eval"]
      return per_eval * count, os.path.relpath(path, ROOT)
  return None, None


def rocprof_kernel_ms(eng, m, model):
  """Per-dispatch average duration (ms) of the hot-path kernels from the newest committed
  rocprofv3 --kernel-trace --stats summary (tools/rocprof_summary.py) of the same generated
  source as this run's kernel, summed over the kernels of one launch, else (None, None)."""
  import glob
  from mujoco_inversedynamicstest_amd import codegen
  if not eng.fast_kernel:
    return None, None
  sha = codegen.source_hash(m, eng.fast_kernel)
  for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "rocprof_bench.json")),
                     reverse=True):
    rec = json.load(open(path))
    if rec.get("model") == model and rec.get("source_sha") == sha:
      return rec["launch_ms"], os.path.relpath(path, ROOT)
  return None, None


def cpu_baseline(m, args):
  """The oracle (kind "port": the CPU restatement of the reference's mj_inverse) compiled for
  this host's CPU at -O3 -march=native, on every core available to the process, one thread per
  core over dynamic chunks (or_inverseBatch). One warm-up pass, then the median of five timed
  passes over the same bounded sample (BASELINE.md's CPU plan)."""
  from mujoco_inversedynamicstest_amd.sampler import sample_states
  from oracle.oracle import Oracle, native_baseline_lib
  nthread = args.cpu_threads or available_cores()
  n = args.cpu_sample or 150_000 * nthread
  cq, cv, ca = sample_states(m, n, first=0)
  o = Oracle(m)
  L, flags = native_baseline_lib()
  warm = max(n // 10, nthread)
  o.inverse_batch(cq[:warm], cv[:warm], ca[:warm], nthread=nthread, lib=L)
  secs = sorted(o.inverse_batch(cq, cv, ca, nthread=nthread, lib=L)[1] for _ in range(5))
  # the baseline build must compute what the checker build computes
  k = min(n, 2048)
  same = bool(np.array_equal(o.inverse_batch(cq[:k], cv[:k], ca[:k], lib=L)[0],
                             o.inverse_batch(cq[:k], cv[:k], ca[:k])[0]))
  med = secs[2]
  return {"value": n / med, "unit": "evals/s", "cores": nthread, "kind": "port",
          "sample": f"{n} humanoid states (first {n} of the same sampler stream), {nthread} "
                    f"threads (cores available to the process: {available_cores()}, "
                    f"os.cpu_count {os.cpu_count()}), oracle/mj_oracle.c {flags}; one warm-up "
                    f"pass of {warm}, median of 5 passes: {med:.3f} s wall "
                    f"(min {secs[0]:.3f}, max {secs[-1]:.3f}); bit-identical to the checker "
                    f"build on the first {k}: {same}"}


def timed(fn, steps, world, dist, torch, dev):
  """Run fn `steps` times between barrier + device syncs; max wall time over ranks (s)."""
  torch.cuda.synchronize(dev)
  if world > 1:
    dist.barrier()
  torch.cuda.synchronize(dev)
  t0 = time.perf_counter()
  for _ in range(steps):
    fn()
  torch.cuda.synchronize(dev)
  if world > 1:
    dist.barrier()
  torch.cuda.synchronize(dev)
  t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
  if world > 1:
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
  return float(t.item())


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--gpus", type=int, default=1)
  ap.add_argument("--steps", type=int, default=200)
  ap.add_argument("--warmup", type=int, default=20)
  ap.add_argument("--batch", type=int, default=65536, help="instances per GPU (weak scaling)")
  ap.add_argument("--global-batch", type=int, default=None,
                  help="total instances over all GPUs (strong scaling; config 3: 262144)")
  ap.add_argument("--model", default="humanoid")
  ap.add_argument("--cpu-threads", type=int, default=None,
                  help="CPU-baseline threads (default: every core available to the process)")
  ap.add_argument("--cpu-sample", type=int, default=None,
                  help="instances in the CPU-baseline sample (rank 0, N=1 only; default "
                       "150k per thread, about 2-3 s of CPU work per thread)")
  ap.add_argument("--no-cpu", action="store_true")
  ap.add_argument("--own-stream", action="store_true",
                  help="config 5: keep the context's own stream (ordered with torch's by "
                       "events around every call) instead of running it on torch's stream")
  ap.add_argument("--config-batch", type=int, default=None,
                  help="batch for --config 4 (default 4096) or base states for 5 (1024)")
  ap.add_argument("--config", type=int, default=2, choices=(2, 4, 5),
                  help="2: the metric's workload (default; with --global-batch 262144 and "
                       "--gpus 8 it is config 3). 4: contacts, keyframe poses, batch 4096. "
                       "5: mjd_inverseFD over 1024 base states. Configs 4/5 are parity cases "
                       "reported for reference (DESIGN.md), not the metric")
  args = ap.parse_args()
  if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
    sys.exit(spawn_ranks(args.gpus))
  if args.config != 2:
    return other_config(args)

  import torch
  import torch.distributed as dist

  world = int(os.environ.get("WORLD_SIZE", "1"))
  rank = int(os.environ.get("RANK", "0"))
  local = int(os.environ.get("LOCAL_RANK", "0"))
  if world != args.gpus:
    raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
  torch.cuda.set_device(local)
  dev = torch.device("cuda", local)
  if world > 1:
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

  from mujoco_inversedynamicstest_amd import codegen, engine, models, parallel
  from mujoco_inversedynamicstest_amd.sampler import sample_states

  m = models.load(args.model, disable_contact=True)
  strong = args.global_batch is not None
  total = args.global_batch if strong else args.batch * world
  first, count = parallel.shard(total, world, rank)
  counts = parallel.shard_counts(total, world)
  q, v, a = sample_states(m, count, first=first)
  eng = engine.InverseEngine(m, capacity=count, device=local)
  eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
  eng.upload_states(q, v, a)
  out = torch.empty((count, m.nv), dtype=torch.float64, device=dev)

  def step():
    eng.inverse(count, out=out, mirror_input=True)

  def step_gather():
    step()
    parallel.gather_to_rank0(out, world, rank, counts)

  for _ in range(args.warmup):
    step()
  elapsed = timed(step, args.steps, world, dist, torch, dev)
  # the same steps followed by the gather of every rank's qfrc_inverse to rank 0
  step_gather()
  elapsed_g = timed(step_gather, args.steps, world, dist, torch, dev)

  # kernel-only average launch time (HIP events on the context's stream) for the roofline
  kernel_ms = eng.time_kernel(count, reps=max(args.steps, 10))
  generic_ms = eng.time_kernel(count, reps=5, generic=True)
  bytes_per_eval = engine.output_bytes_per_eval(m)
  achieved = bytes_per_eval * count / (kernel_ms * 1e-3) / 1e9
  traffic, traffic_src = pmc_traffic(eng, m, args.model, count)
  prof_ms, prof_src = rocprof_kernel_ms(eng, m, args.model)
  if prof_ms is not None and count != 65536:
    prof_ms = None        # the committed summary is of the 65,536 launch

  # every rank's full qfrc_inverse on rank 0 (outside the timed regions): a checksum of
  # checksums over the whole global batch, and a spot check of the gathered rows
  gathered = parallel.gather_to_rank0(out, world, rank, counts)
  torch.cuda.synchronize(dev)
  checksum = None
  if rank == 0:
    full = torch.cat(gathered)
    assert full.shape == (total, m.nv)
    checksum = float(full.abs().sum(dim=1).sum())

  cpu = None
  if rank == 0 and world == 1 and not args.no_cpu:
    cpu = cpu_baseline(m, args)

  if rank == 0:
    value = total * args.steps / elapsed
    rec = {
        "metric": METRIC,
        "value": value,
        "unit": "evals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: config-2 sampler (seed 20250314), inputs resident in HBM",
        "config": {"workload": f"{args.model} 27-DoF mj_inverse (skipstage NONE), contacts "
                               f"disabled, nefc=0, full mjData mirror written",
                   "per_gpu_batch": count, "global_batch": total,
                   "parallelism": f"dp{world}"},
        "with_gather": {"value": total * args.steps / elapsed_g,
                        "ms_per_step": elapsed_g / args.steps * 1e3,
                        "bytes_to_rank0_per_step": 8 * m.nv * (total - counts[0]),
                        "collective": "RCCL point-to-point sends of qfrc_inverse to rank 0"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic,
                     "traffic_unit": "bytes per launch", "traffic_source": traffic_src,
                     "traffic_ratio": (traffic / (bytes_per_eval * count)) if traffic else None,
                     "algorithmic_bytes_per_launch": bytes_per_eval * count,
                     "kernel": ("+".join(codegen.hot_kernels(eng.fast_kernel)
                                         + [eng.constraint_kernel])
                                if eng.fast_kernel else "k_inverse<0>"),
                     "kernel_ms": kernel_ms,
                     "kernel_ms_method": "HIP events on the context's stream around `reps` "
                                         "back-to-back launches of the hot path, divided by "
                                         "reps (rocprof's per-dispatch durations each include "
                                         "their own dispatch ramp, so their sum reads a few "
                                         "us higher)",
                     "rocprof_kernel_ms": prof_ms,
                     "rocprof_source": prof_src,
                     "frac_rocprof": (bytes_per_eval * count / (prof_ms * 1e-3) / 1e9
                                      / HBM_PEAK_GBPS if prof_ms else None),
                     "generic_kernel_ms": generic_ms,
                     "bytes_per_eval": bytes_per_eval},
        "cpu_baseline": cpu,
        "checksum_qfrc_inverse": checksum,
    }
    print(json.dumps(rec), flush=True)
  eng.close()
  if world > 1:
    dist.destroy_process_group()


def other_config(args):
  """Throughput of configs 4 (contacts) and 5 (finite-difference Jacobians), 1 GPU."""
  import torch
  from mujoco_inversedynamicstest_amd import codegen, engine, models
  from mujoco_inversedynamicstest_amd.sampler import sample_contact_states
  if args.config == 5:
    return config5(args)
  torch.cuda.set_device(0)
  m = models.load(args.model, disable_contact=False)
  B = args.config_batch or 4096
  q, v, a = sample_contact_states(m, B)
  eng = engine.InverseEngine(m, capacity=B)
  eng.upload_states(q, v, a)
  for _ in range(args.warmup):
    eng.inverse(B, mirror_input=True)
  torch.cuda.synchronize()
  t0 = time.perf_counter()
  for _ in range(args.steps):
    eng.inverse(B, mirror_input=True)
  torch.cuda.synchronize()
  dt = (time.perf_counter() - t0) / args.steps
  kernel_ms = eng.time_kernel(B, reps=max(args.steps, 10))
  ncon = eng.field_int("con_count", 0, B)[:, 0]
  nefc = eng.field_int("efc_count", 0, B)[:, 0]
  # algorithmic bytes of one launch: B_eval per instance plus the rows and contacts this
  # batch actually produced (engine.constraint_bytes)
  base = engine.output_bytes_per_eval(m) * B
  extra = engine.constraint_bytes(m, nefc.sum(), ncon.sum(), B)
  achieved = (base + extra) / (kernel_ms * 1e-3) / 1e9
  traffic, traffic_src = pmc_traffic(eng, m, "humanoid_contact", B, "pmc_traffic_c4.json")
  rec = {"metric": "mj_inverse evals/sec, config 4 (contacts on)", "value": B / dt,
         "unit": "evals/s", "n_gpus": 1, "steps": args.steps, "ms_per_step": dt * 1e3,
         "kernel_ms": kernel_ms, "dtype": "f64",
         "kernel": (f"generated {'+'.join(codegen.hot_kernels(eng.fast_kernel))} + "
                    f"{eng.constraint_kernel}" if eng.fast_kernel
                    else "k_inverse<0, contacts> (generic)"),
         "config": {"workload": f"{args.model} keyframe poses + noise, contacts on",
                    "batch": B},
         "ncon_hist": np.bincount(ncon).tolist(), "nefc_max": int(nefc.max()),
         "nefc_mean": float(nefc.mean()),
         "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS,
                      "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic,
                      "traffic_unit": "bytes per launch", "traffic_source": traffic_src,
                      "traffic_ratio": (traffic / (base + extra)) if traffic else None,
                      "algorithmic_bytes_per_launch": base + extra,
                      "bytes_detail": {"b_eval_per_instance": engine.output_bytes_per_eval(m),
                                       "rows": int(nefc.sum()), "contacts": int(ncon.sum()),
                                       "constraint_bytes": extra},
                      "kernel_ms": kernel_ms,
                      "kernel_ms_method": "HIP events on the context's stream around reps "
                                          "back-to-back launches of every kernel of one call"}}
  print(json.dumps(rec), flush=True)
  eng.close()


def config5(args):
  """Config 5: batched mjd_inverseFD over base states resident in HBM, one process per GPU.

  Each rank owns a contiguous shard of the global base-state set (weak scaling: --config-batch
  base states per GPU, default 1024), so all 3nv+1 perturbations of a base state and their
  differencing stay on one GPU. A step is one mjd_inverseFD over the shard:
  expand, mj_inverse over every perturbation, difference, Jacobians left in HBM. After timing,
  rank 0 gathers every rank's DfDq/DfDv/DfDa over RCCL (timed separately), and the
  PCIe-inclusive host-array rate is measured once for reference."""
  import torch
  import torch.distributed as dist
  from mujoco_inversedynamicstest_amd import engine, models, parallel
  from mujoco_inversedynamicstest_amd.sampler import sample_states
  world = int(os.environ.get("WORLD_SIZE", "1"))
  rank = int(os.environ.get("RANK", "0"))
  local = int(os.environ.get("LOCAL_RANK", "0"))
  if world != args.gpus:
    raise SystemExit(f"bench.py --config 5: --gpus {args.gpus} but WORLD_SIZE={world}")
  torch.cuda.set_device(local)
  dev = torch.device("cuda", local)
  if world > 1:
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
  m = models.load(args.model, disable_contact=True)
  nb = args.config_batch or 1024
  P = 3 * m.nv + 1
  first, count = parallel.shard(nb * world, world, rank)
  q, v, a = sample_states(m, count, first=first)
  eng = engine.InverseEngine(m, capacity=count * P, device=local)
  if not args.own_stream:
    # the context runs on torch's stream: no cross-stream event waits around each call
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
  tq, tv, ta = (torch.from_numpy(x).to(dev) for x in (q, v, a))
  mk = lambda: torch.empty((count, m.nv, m.nv), dtype=torch.float64, device=dev)
  out = (mk(), mk(), mk(), None)
  torch.cuda.synchronize(dev)

  def step():
    eng.inverse_fd(tq, tv, ta, out=out)

  for _ in range(args.warmup):
    step()
  dt = timed(step, args.steps, world, dist, torch, dev) / args.steps
  # gather of the Jacobians to rank 0 (RCCL point-to-point), outside the timed region
  jac = torch.stack(out[:3])
  torch.cuda.synchronize(dev)
  g0 = time.perf_counter()
  gathered = parallel.gather_to_rank0(jac, world, rank)
  torch.cuda.synchronize(dev)
  gather_ms = (time.perf_counter() - g0) * 1e3
  # PCIe-inclusive reference: host arrays in, host Jacobians out, one call
  h0 = time.perf_counter()
  eng.inverse_fd(q, v, a)
  host_dt = time.perf_counter() - h0
  if rank == 0:
    checksum = float(sum(float(x.abs().sum()) for x in gathered))
    rec = {"metric": "mjd_inverseFD Jacobian sets/sec, config 5", "value": world * count / dt,
           "unit": "base states/s", "inverse_evals_per_s": world * count * P / dt,
           "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": dt * 1e3, "higher_is_better": True, "scaling": "weak",
           "dtype": "f64", "data": "synthetic: config-2 sampler, base states resident in HBM",
           "config": {"workload": f"{args.model} mjd_inverseFD, {count} base states per GPU x "
                                  f"{P} evaluations (DfDq, DfDv, DfDa, forward differences, "
                                  f"eps 1e-6), Jacobians left in HBM",
                      "per_gpu_base_states": count, "global_base_states": world * count,
                      "parallelism": f"dp{world}"},
           "gather_to_rank0_ms": gather_ms,
           "pcie_inclusive_rank0_base_states_per_s": count / host_dt,
           "checksum_jacobians": checksum}
    print(json.dumps(rec), flush=True)
  eng.close()
  if world > 1:
    dist.destroy_process_group()


if __name__ == "__main__":
  main()
