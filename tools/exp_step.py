"""Performance experiment (not part of the product): per-step time of the headline workload
under different call variants (GPU box).

  python tools/exp_step.py [steps]

Prints ms per step for: the C-side timing loop (mjhip_timeInverseKernel), the Python call
with and without the row-major qfrc_inverse output, on the context's own stream and on
torch's current stream.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(steps=500):
  import torch
  from mujoco_inversedynamicstest_amd import engine, models
  from mujoco_inversedynamicstest_amd.sampler import sample_states
  torch.cuda.set_device(0)
  m = models.load("humanoid", disable_contact=True)
  B = 65536
  q, v, a = sample_states(m, B)
  eng = engine.InverseEngine(m, capacity=B)
  eng.upload_states(q, v, a)
  out = torch.empty((B, m.nv), dtype=torch.float64, device="cuda:0")

  def timed(fn, label):
    for _ in range(50):
      fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
      fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    print(f"{label:44s} {dt*1e3:8.4f} ms/step", flush=True)

  print(f"C timing loop (timeInverseKernel)            {eng.time_kernel(B, reps=steps):8.4f}")
  timed(lambda: eng.inverse(B, mirror_input=True), "context stream, no row-major out")
  timed(lambda: eng.inverse(B, out=out, mirror_input=True), "context stream, row-major out")
  eng.set_stream(torch.cuda.current_stream().cuda_stream)
  print(f"torch stream handle: {torch.cuda.current_stream().cuda_stream}")
  print(f"C timing loop on torch stream                {eng.time_kernel(B, reps=steps):8.4f}")
  timed(lambda: eng.inverse(B, mirror_input=True), "torch stream, no row-major out")
  timed(lambda: eng.inverse(B, out=out, mirror_input=True), "torch stream, row-major out")
  t0 = time.perf_counter()
  for _ in range(steps):
    eng.inverse(B, out=out, mirror_input=True)
  t_issue = (time.perf_counter() - t0) / steps
  torch.cuda.synchronize()
  print(f"host issue time per step (no sync)           {t_issue*1e3:8.4f}")
  eng.close()


if __name__ == "__main__":
  main(int(sys.argv[1]) if len(sys.argv) > 1 else 500)
