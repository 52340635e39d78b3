"""Make the rne_post golden fixtures (run in the build container; /root/reference is absent
on the GPU box, which reads only the outputs).

The reference's only numeric expectations on the mj_inverse -> mj_rnePostConstraint path are
the force/torque readings written into the `user` attribute of each sensor of the 15 models
under test/engine/testdata/core_smooth/rne_post/{connect,weld}/ (checked at static
equilibrium by TestConnect / TestWeld, test/engine/engine_core_smooth_test.cc:165-303).

For every model this script writes
  tests/golden/rne_post/<dir>_<name>.npz   the model compiled by mjcf.py (data, not source)
  tests/golden/rne_post.json              per model: the reference test that reads it, which
                                          sensor values that test checks, and the expected
                                          values (the sensors' `user` attributes)

    python tests/golden/make_rne_post.py [--reference /root/reference]
"""
import argparse
import glob
import json
import os
import sys
import xml.etree.ElementTree as ET

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from mujoco_inversedynamicstest_amd import mjcf  # noqa: E402

REL = "test/engine/testdata/core_smooth/rne_post"
# engine_core_smooth_test.cc: which driver each model runs under, and the TEST_F's line.
# TestConnect checks sensordata[0:3] against sensor_user[0:3]; TestWeld checks the first three
# values of every sensor. force_torque_free_rotated_tendon.xml has no TEST_F of its own.
TESTS = {
    "connect/force_slide": ("TestConnect", 182), "connect/force_slide_rotated": ("TestConnect", 189),
    "connect/force_free": ("TestConnect", 196), "connect/torque_free": ("TestConnect", 203),
    "connect/multiple_constraints": ("TestConnect", 210),
    "weld/force_free": ("TestWeld", 242), "weld/force_free_rotated": ("TestWeld", 249),
    "weld/force_torque_free": ("TestWeld", 256),
    "weld/force_torque_free_rotated": ("TestWeld", 263),
    "weld/force_torque_free_rotated_tendon": ("TestWeld", None),
    "weld/tfratio0_force_free": ("TestConnect", 270),
    "weld/tfratio0_force_slide": ("TestConnect", 277),
    "weld/tfratio0_torque_free": ("TestConnect", 284),
    "weld/tfratio0_force_slide_rotated": ("TestConnect", 291),
    "weld/tfratio0_multiple_constraints": ("TestConnect", 298),
}


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--reference", default="/root/reference")
  args = ap.parse_args()
  cases = {}
  files = sorted(glob.glob(os.path.join(args.reference, REL, "*", "*.xml")))
  assert len(files) == len(TESTS), files
  for path in files:
    key = os.path.relpath(path, os.path.join(args.reference, REL))[:-4]
    driver, line = TESTS[key]
    m = mjcf.load_xml(path)
    name = key.replace("/", "_")
    m.save(os.path.join(HERE, "rne_post", name + ".npz"))
    users = [[float(x) for x in s.get("user").split()]
             for s in ET.parse(path).getroot().find("sensor")]
    if driver == "TestConnect":      # sensordata[0:3] vs sensor_user[0:3]
      checks = [[0, users[0][:3]]]
    else:                            # every sensor: sensordata[adr + i] vs its user[i], i < 3
      checks = [[int(m.sensor_adr[s]), users[s][:3]] for s in range(len(users))]
    cases[name] = {"source": f"{REL}/{key}.xml", "driver": driver,
                   "test": f"test/engine/engine_core_smooth_test.cc:{line}" if line else None,
                   "checks": checks}
    print(name, driver, checks)
  with open(os.path.join(HERE, "rne_post.json"), "w") as f:
    json.dump(cases, f, indent=1)


if __name__ == "__main__":
  main()
