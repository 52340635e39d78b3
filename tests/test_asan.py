"""Sanitizer run of the CPU code (oracle/mj_oracle.c and the host compilation of the device
pipeline, tests/cpu_kernel_harness.cpp) under AddressSanitizer + UndefinedBehaviorSanitizer.

GPU sanitizers are not available on the MI355X pool, so the device code is checked through
its host compilation: the same engine_device.h source, on the same models and states the
CPU suite uses (tests/asan_driver.py, in a child process with libasan preloaded)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _runtime(name):
  p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True)
  path = p.stdout.strip()
  return path if os.path.isabs(path) and os.path.exists(path) else None


@pytest.mark.timeout(900)
def test_oracle_and_host_device_build_under_asan_ubsan():
  asan, ubsan = _runtime("libasan.so"), _runtime("libubsan.so")
  if not asan or not ubsan:
    pytest.skip("gcc sanitizer runtimes not installed")
  subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)
  env = dict(os.environ)
  env.update(
      LD_PRELOAD=f"{asan}:{ubsan}",
      ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:verify_asan_link_order=0",
      UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
      ORACLE_LIB=os.path.join(ROOT, "oracle", "liboracle_asan.so"),
      KERNEL_HARNESS_FLAGS="-O1 -g -fsanitize=address,undefined -fno-sanitize-recover=undefined "
                           "-fno-omit-frame-pointer")
  r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "asan_driver.py")], env=env,
                     capture_output=True, text=True, timeout=880)
  tail = (r.stdout + r.stderr)[-6000:]
  assert r.returncode == 0, tail
  assert "ASAN_DRIVER_OK" in r.stdout, tail
  assert "runtime error" not in r.stderr, tail
