"""Compile the reference's MJCF models into the bundled .npz files.

Run in the build container (the only place /root/reference exists):
    python tools/compile_models.py [--reference /root/reference]
The outputs (mujoco_inversedynamicstest_amd/models/*.npz) are committed, so the GPU box
never needs the reference.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mujoco_inversedynamicstest_amd import mjcf, models  # noqa: E402


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--reference", default="/root/reference")
  args = ap.parse_args()
  for name, rel in models.SOURCES.items():
    src = os.path.join(args.reference, rel)
    m = mjcf.load_xml(src)
    m.save(models.path(name))
    print(f"{name}: {rel} -> {models.path(name)} (nq={m.nq} nv={m.nv} nbody={m.nbody})")


if __name__ == "__main__":
  main()
