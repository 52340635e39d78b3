"""Measurement experiment (not part of the product): where bench.py's step time goes beyond
the kernel time of the roofline line. Times, over the same mirror-resident 65,536 humanoid
states: the kernels alone (mjhip_timeInverseKernel), the Python step with and without the
qfrc_inverse output tensor (wall clock over back-to-back steps and HIP events on the stream),
and the step's host-side cost (the same calls with the GPU idle-synchronized per call).

  python tools/exp_step.py          # GPU box
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
  import torch
  from mujoco_inversedynamicstest_amd import engine, models
  from mujoco_inversedynamicstest_amd.sampler import sample_states
  dev = torch.device("cuda", 0)
  m = models.load("humanoid", disable_contact=True)
  B = 65536
  q, v, a = sample_states(m, B)
  e = engine.InverseEngine(m, capacity=B)
  e.set_stream(torch.cuda.current_stream(dev).cuda_stream)
  e.upload_states(q, v, a)
  out = torch.empty((B, m.nv), dtype=torch.float64, device=dev)
  steps = 200

  def wall(fn):
    for _ in range(5):
      fn()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(steps):
      fn()
    ev1.record()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / steps * 1e3, ev0.elapsed_time(ev1) / steps

  with_out = lambda: e.inverse(B, out=out, mirror_input=True)
  no_out = lambda: e.inverse(B, mirror_input=True)
  for rep in range(2):
    k = e.time_kernel(B, reps=steps)
    w1, ev1 = wall(with_out)
    w2, ev2 = wall(no_out)
    t0 = time.perf_counter()
    for _ in range(50):
      with_out()
    host = (time.perf_counter() - t0) / 50 * 1e3
    torch.cuda.synchronize(dev)
    print(f"rep {rep}: kernels {k*1e3:.1f} us | step with out: wall {w1*1e3:.1f} us, events "
          f"{ev1*1e3:.1f} us | step without out: wall {w2*1e3:.1f} us, events {ev2*1e3:.1f} us "
          f"| host-side submit cost per step {host*1e3:.1f} us", flush=True)
  e.close()


if __name__ == "__main__":
  main()
