"""raytracer::camera (src/camera.hxx:19-77) over the C-ABI.

The basis is computed by the library's host code with the reference constructor's float
operations (rt_camera_init), so the kernel receives bit-identical inputs.
"""
import ctypes as C

from . import _abi as abi
from ._lib import check, lib

REFERENCE = abi.RT_CAMERA_REFERENCE  # camera::ray as shipped (direction omits "- origin")
CORRECTED = abi.RT_CAMERA_CORRECTED  # direction - origin


class Camera:
    """camera(position, lookat, up, aspect, vFOV, aperture, focus_distance), camera.hxx:24-44."""

    def __init__(self, position, lookat, up, aspect, vfov, aperture, focus_distance, mode=REFERENCE):
        f3 = C.c_float * 3
        self.c = abi.RtCamera()
        check(lib().rt_camera_init(f3(*position), f3(*lookat), f3(*up), aspect, vfov, aperture,
                                   focus_distance, mode, C.byref(self.c)))

    @classmethod
    def default(cls, width, height, mode=REFERENCE):
        """The camera main() builds for a width x height image (src/main.cxx:179-183)."""
        self = cls.__new__(cls)
        self.c = abi.RtCamera()
        check(lib().rt_camera_default(width, height, mode, C.byref(self.c)))
        return self

    @classmethod
    def cuda(cls, width, height):
        """The reference CUDA variant's camera (src/CUDA/cuda_impl.cu:371-375)."""
        self = cls.__new__(cls)
        self.c = abi.RtCamera()
        check(lib().rt_camera_cuda(width, height, C.byref(self.c)))
        return self

    @property
    def mode(self):
        return self.c.mode

    def basis(self):
        c = self.c
        return {"origin": tuple(c.origin), "lower_left_corner": tuple(c.lower_left_corner),
                "horizontal": tuple(c.horizontal), "vertical": tuple(c.vertical),
                "lens_radius": c.lens_radius, "mode": c.mode}
