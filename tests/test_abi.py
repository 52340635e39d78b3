"""The C-ABI library loads and exports every symbol include/mjhip.h declares (no GPU)."""
import ctypes
import os
import re
import subprocess

import pytest

from mujoco_inversedynamicstest_amd import engine, fields, host, models

HEADER = os.path.join(fields.INCLUDE_DIR, "mjhip.h")


def declared_symbols():
  text = open(HEADER).read()
  return sorted(set(re.findall(r"MJHIP_API\s+[\w\s\*]+?\b(mjhip_\w+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
  assert os.path.exists(engine.LIB_PATH), "run __graft_entry__.build() first"
  out = subprocess.run(["nm", "-D", "--defined-only", engine.LIB_PATH], capture_output=True,
                       text=True, check=True).stdout
  exported = set(re.findall(r"\bT (mjhip_\w+)", out))
  decl = declared_symbols()
  assert len(decl) >= 25
  missing = [s for s in decl if s not in exported]
  assert not missing, missing


def test_python_binding_covers_header():
  assert sorted(engine.SIGNATURES) == declared_symbols()
  engine.lib()   # binds every signature


def test_ctypes_struct_sizes_match_c():
  """sizeof(mjhipModel/mjhipData) seen by C equals the ctypes mirrors (compiled probe)."""
  src = ('#include "mjhip.h"\n#include <stdio.h>\n'
         'int main(){printf("%zu %zu %zu\\n", sizeof(mjhipModel), sizeof(mjhipData),'
         ' sizeof(mjhipOption));}')
  build = os.path.join(os.path.dirname(__file__), "_build")
  os.makedirs(build, exist_ok=True)
  c = os.path.join(build, "probe.c")
  exe = os.path.join(build, "probe")
  open(c, "w").write(src)
  subprocess.run(["gcc", "-I", fields.INCLUDE_DIR, "-o", exe, c], check=True)
  sm, sd, so = map(int, subprocess.run([exe], capture_output=True, text=True,
                                       check=True).stdout.split())
  assert sm == ctypes.sizeof(fields.CModel)
  assert sd == ctypes.sizeof(fields.CData)
  assert so == ctypes.sizeof(fields.Option)


def test_output_doubles_abi(humanoid):
  L = engine.lib()
  cm = host.model_struct(humanoid)
  assert L.mjhip_outputDoubles(ctypes.byref(cm)) == 2563
  assert L.mjhip_fieldSize(ctypes.byref(cm), b"qM") == 243
  assert L.mjhip_fieldSize(ctypes.byref(cm), b"nope") == -1


def test_no_cpu_fallback_without_device(humanoid):
  """Without a GPU the engine fails loudly (MJHIP_ERR_NO_DEVICE), it never computes on CPU."""
  if engine.lib().mjhip_deviceCount() > 0:
    pytest.skip("a GPU is present")
  with pytest.raises(engine.MJHIPError, match="NO_DEVICE"):
    engine.InverseEngine(humanoid, capacity=64)


@pytest.mark.gpu
def test_unsupported_model_rejected():
  """A model outside the device subset (here: mjENBL_INVDISCRETE with RK4, an mjERROR in
  the reference) is rejected at context creation with MJHIP_ERR_MODEL, never run
  approximately (the rejection happens after the device check, so this needs the GPU)."""
  m = models.load("humanoid")
  m.opt["enableflags"] |= 1 << 3
  m.opt["integrator"] = 1
  with pytest.raises(engine.MJHIPError, match="MODEL"):
    engine.InverseEngine(m, capacity=64)


def test_mjdata_row_buffers_sized_by_model_capacity():
  """MjData's efc_* / con_* buffers come from mjhip_modelCapacity (no GPU needed), the same
  bounds the oracle computes for its own rows."""
  import ctypes
  from mujoco_inversedynamicstest_amd import fields, host, models
  from oracle.oracle import lib as olib
  for name, contacts in (("humanoid", True), ("humanoid", False), ("inverse_test", False)):
    m = models.load(name, disable_contact=not contacts)
    rows, cons = host.model_capacity(m)
    cm = host.model_struct(m)
    assert rows == olib().or_efcCapacity(ctypes.byref(cm))
    assert cons == max(olib().or_contactCapacity(ctypes.byref(cm)), 0)
    d = host.MjData(m)
    assert d.struct.efc_capacity == rows and d.struct.con_capacity == cons
    for f in fields.EFC_FIELDS:
      assert d._rows[f.name].size == max(rows * f.row_size(m.sizes), 1)
    assert d.efc("efc_J").shape == (0, m.nv)
