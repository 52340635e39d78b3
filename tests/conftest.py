"""Shared fixtures. GPU tests are marked `gpu`; everything else runs on CPU (no GPU here)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
  sys.path.insert(0, ROOT)

from mujoco_inversedynamicstest_amd import models as _models  # noqa: E402


def pytest_configure(config):
  config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")


@pytest.fixture(scope="session")
def humanoid():
  """humanoid.xml with contacts disabled (config 2 of BASELINE.json)."""
  return _models.load("humanoid", disable_contact=True)


@pytest.fixture(scope="session")
def humanoid_contacts():
  return _models.load("humanoid")


@pytest.fixture(scope="session")
def arm2():
  """src/inverse/test.xml, the model of the reference's inverse_test.cpp driver."""
  return _models.load("inverse_test", disable_contact=True)


@pytest.fixture(scope="session")
def linear():
  return _models.load("linear", disable_contact=True)


@pytest.fixture(scope="session")
def inertia():
  return _models.load("inertia", disable_contact=True)


@pytest.fixture
def rng():
  return np.random.default_rng(20250314)
