"""Performance experiment (not part of the product): A/B variants of the straight-line humanoid
kernel without rebuilding libmjhip.so.

  python tools/exp_variants.py            # build the variants' code objects (no GPU needed)
  python tools/exp_variants.py run        # GPU box: time each against the bundled kernel

Each variant is the run-time specialized kernel (specialize.py) generated with some codegen
knobs changed; the run loads it into a context (mjhip_contextLoadKernel), checks that its
qfrc_inverse equals the bundled kernel's bit for bit, and times REPS launches with HIP events
(mjhip_timeInverseKernel) at batch 65,536, interleaved with the bundled kernel.
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tools", "exp_lib", "variants")

# name -> codegen attribute overrides
VARIANTS = {
    "control": {},
    "every_reread_temporal": {"NT_TEMPORAL": {"qM", "cdof", "cinert", "qacc", "qfrc_passive",
                                              "qpos", "qvel", "ten_length"}},
    "va_nt_loads": {"NT_LOAD_STAGES": ("va",)},
}


def _model():
  from mujoco_inversedynamicstest_amd import models
  return models.load("humanoid", disable_contact=True)


def build():
  from mujoco_inversedynamicstest_amd import codegen, specialize
  os.makedirs(OUT, exist_ok=True)
  m = _model()
  index = {}
  for name, over in VARIANTS.items():
    saved = {k: getattr(codegen, k) for k in over}
    try:
      for k, v in over.items():
        setattr(codegen, k, v)
      image, kname, sig, cmode = specialize.code_object(m)
    finally:
      for k, v in saved.items():
        setattr(codegen, k, v)
    path = os.path.join(OUT, f"{name}.hsaco")
    with open(path, "wb") as f:
      f.write(image)
    index[name] = {"kernel": kname, "sig": sig, "cmode": cmode}
    print(f"{name}: {kname} {len(image)} bytes")
  with open(os.path.join(OUT, "index.json"), "w") as f:
    json.dump(index, f, indent=1)


def run(B=65536, reps=50, rounds=3):
  import numpy as np
  from mujoco_inversedynamicstest_amd import engine
  from mujoco_inversedynamicstest_amd.sampler import sample_states
  index = json.load(open(os.path.join(OUT, "index.json")))
  m = _model()
  q, v, a = sample_states(m, B)
  base = engine.InverseEngine(m, capacity=B, specialize=False)
  assert base.fast_kernel == "humanoid"
  ref = base.inverse(q, v, a)
  base.upload_states(q, v, a)
  engines = {}
  for name, rec in index.items():
    e = engine.InverseEngine(m, capacity=B, specialize=False)
    image = open(os.path.join(OUT, f"{name}.hsaco"), "rb").read()
    buf = ctypes.create_string_buffer(image, len(image))
    engine._check(engine.lib().mjhip_contextLoadKernel(e.ctx, buf, len(image),
                                                       rec["kernel"].encode(),
                                                       ctypes.c_ulonglong(rec["sig"]),
                                                       rec["cmode"]), "load")
    out = e.inverse(q, v, a)
    same = bool(np.array_equal(out, ref))
    e.upload_states(q, v, a)
    engines[name] = (e, same)
  times = {name: [] for name in ["bundled"] + list(engines)}
  for _ in range(rounds):
    times["bundled"].append(base.time_kernel(B, reps))
    for name, (e, _) in engines.items():
      times[name].append(e.time_kernel(B, reps))
  for name, t in times.items():
    same = engines[name][1] if name in engines else True
    print(f"{name:20s} {min(t)*1e3:8.1f} us (median {np.median(t)*1e3:8.1f})  "
          f"bit-identical {same}", flush=True)
  for e, _ in engines.values():
    e.close()
  base.close()


if __name__ == "__main__":
  if len(sys.argv) > 1 and sys.argv[1] == "run":
    for b in os.environ.get("VARIANT_B", "65536").split(","):
      print(f"== batch {b}", flush=True)
      run(B=int(b))
  else:
    build()
