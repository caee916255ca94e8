"""MI355X-native path tracer: the per-pixel render loop of Alabuta/RaytracingInOneWeekend
(app::color -> raytracer::hit_world -> raytracer::apply_material) as a HIP megakernel for
gfx950 behind a C ABI (include/rt_api.h). See DESIGN.md.
"""
from . import _abi as abi  # noqa: F401
from ._lib import RtError, lib  # noqa: F401
from .camera import CORRECTED, REFERENCE, Camera  # noqa: F401
from .render import (DeviceScene, MultiContext, default_options, default_options_set,  # noqa: F401
                     epilogue_rgb8_device, make_params, options, parse_options, render_cuda_impl, render_f32,
                     release_cached, render_multi_f32, render_multi_rgb8, render_rgb8, save_ppm,
                     set_default_options, tile_order)
from .scene import (Dielectric, Lambert, Metal, RaytracerData, Sphere, cuda_scene_arrays, huge_scene,  # noqa: F401
                    huge_scene_arrays, simple_scene, simple_scene_arrays)

__version__ = "0.1.0"
