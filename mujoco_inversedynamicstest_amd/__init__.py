"""mujoco_inversedynamicstest_amd: MI355X-native batched inverse dynamics (mj_inverse).

Host-side mirror of the reference's inverse-dynamics interface
(fancifulland2718/mujoco_InverseDynamicsTest, src/engine/engine_inverse.c) over the
C-ABI library libmjhip.so (include/mjhip.h), whose compute path is hand-written HIP for
gfx950.
"""
from .mjcf import load_xml, load_xml_string, Model, MJCFError  # noqa: F401
