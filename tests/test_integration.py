"""The reference-side adapter (integration/engine_inverse_mjhip.c) compiles against the
reference's real public headers: every mjhipModel/mjhipData field is assigned from the
mjModel/mjData field of the same name, so a name or element-type mismatch with the
reference's layout contract (include/mujoco/mjxmacro.h) is a compile error. Only runs where
the reference tree exists (the build container); nothing is copied from it."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_INC = "/root/reference/include"


@pytest.mark.skipif(not os.path.isdir(REF_INC), reason="reference headers not present")
def test_adapter_compiles_against_reference_headers(tmp_path):
  out = tmp_path / "adapter.o"
  r = subprocess.run(["gcc", "-std=c11", "-c", "-Wall", "-Werror",
                      "-Werror=incompatible-pointer-types", "-Wno-unused-function",
                      "-I", REF_INC, "-I", os.path.join(ROOT, "include"),
                      "-o", str(out), os.path.join(ROOT, "integration", "engine_inverse_mjhip.c")],
                     capture_output=True, text=True)
  assert r.returncode == 0, r.stderr[-3000:]
