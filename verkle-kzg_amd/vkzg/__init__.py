"""vkzg -- MI355X vector-commitment MSM engine (host-side Python handle on libvkzg.so).

The compute path is HIP (libvkzg.so, C ABI include/vc_msm.h); this package only marshals
arguments. Importing it does not touch the GPU.
"""
from ._lib import LIB_PATH, VCError, header_functions, lib  # noqa: F401
from .engine import (CURVE_IDS, NL, SCALAR_R, Engine, arrays_to_points, dot_mod, ints_to_limbs,  # noqa: F401
                     limb_rows_to_ints, limbs_to_int, points_to_arrays, random_base_scalars, random_scalars)
