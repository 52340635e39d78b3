"""Performance experiment (not part of the product): run bench.py against another build of
libmjhip (tools/exp/*.so), e.g. compile-flag variants.

  python tools/exp_lib_bench.py tools/exp/libmjhip_wpe2.so --config 4 --steps 20
"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mujoco_inversedynamicstest_amd import engine  # noqa: E402

engine.LIB_PATH = os.path.abspath(sys.argv[1])
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
