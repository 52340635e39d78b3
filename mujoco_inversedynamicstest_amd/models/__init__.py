"""Bundled compiled models (.npz, produced by tools/compile_models.py from the reference's
MJCF files). They travel with the repo, so nothing reads /root/reference at run time."""
from __future__ import annotations

import os

from ..mjcf import Model

_HERE = os.path.dirname(os.path.abspath(__file__))

# name -> MJCF path relative to the reference root
SOURCES = {
    "humanoid": "model/humanoid/humanoid.xml",                  # BASELINE.json configs 2-5
    # the reference's 627-dof benchmark model: humanoid.xml attached + 100 replicated bodies
    "humanoid100": "model/humanoid/humanoid100.xml",
    "slider_crank": "model/slider_crank/slider_crank.xml",      # BASELINE.json config 1
    "inverse_test": "src/inverse/test.xml",                      # inverse_test.cpp model
    "linear": "test/engine/testdata/derivative/linear.xml",     # LinearSystemInverse
    "inertia": "test/engine/testdata/inertia.xml",              # FactorI / FactorIs
    "weld": "test/engine/testdata/weld.xml",                    # equality: weld variants
    "connect": "test/engine/testdata/connect.xml",              # equality: connect
    "equality_site": "test/engine/testdata/equality_site.xml",  # site-semantic equalities
    # EqualityBodySite (engine_core_constraint_test.cc:253-289)
    "equality_compare": "test/engine/testdata/equality_site_body_compare.xml",
}

mjDSBL_CONTACT = 1 << 4
mjDSBL_SENSOR = 1 << 12


def path(name: str) -> str:
  return os.path.join(_HERE, name + ".npz")


def load(name: str, disable_contact: bool = False, disable_sensor: bool = False) -> Model:
  m = Model.load(path(name))
  if disable_contact:
    m.opt["disableflags"] = int(m.opt["disableflags"]) | mjDSBL_CONTACT
  if disable_sensor:
    m.opt["disableflags"] = int(m.opt["disableflags"]) | mjDSBL_SENSOR
  return m
